"""The device graph helpers (gu_* C-ABI through gym_flock.envs.spatial.utils) against
the reference's recorded outputs (tests/golden/graph_utils.npz) and the oracle. Edge
lists, distances and differences are compared bit-exactly. Needs an MI355X."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import graph_utils as og

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("gym_flock._native")
from gym_flock.envs.spatial import utils as gu  # noqa: E402

G = np.load(os.path.join(GOLDEN, "graph_utils.npz"))
RADIUS = sorted({k[:-5] for k in G.files if k.startswith("radius_") and k.endswith("_pos1")})
KNN = sorted({k[:-5] for k in G.files if k.startswith("k_") and k.endswith("_pos1")})


def same(got, s, q, r, diff):
    (gs, gq), gr, gd = got
    assert gs.dtype == np.intp and gq.dtype == np.intp
    np.testing.assert_array_equal(gs, s)
    np.testing.assert_array_equal(gq, q)
    np.testing.assert_array_equal(gr, r)
    np.testing.assert_array_equal(gd, diff)


@pytest.mark.parametrize("tag", RADIUS)
def test_radius_edges_match_reference(tag):
    p2 = G[tag + "_pos2"] if tag + "_pos2" in G.files else None
    got = gu._get_graph_edges(float(G[tag + "_rad"]), G[tag + "_pos1"], p2, self_loops=bool(G[tag + "_self"]))
    same(got, G[tag + "_snd"], G[tag + "_rcv"], G[tag + "_r"], G[tag + "_diff"])
    assert got[2].shape[1] == 2


@pytest.mark.parametrize("tag", KNN)
def test_k_edges_match_reference(tag):
    p2 = G[tag + "_pos2"] if tag + "_pos2" in G.files else None
    got = gu._get_k_edges(int(G[tag + "_k"]), G[tag + "_pos1"], p2, self_loops=bool(G[tag + "_self"]),
                          allow_nearest=bool(G[tag + "_near"]))
    same(got, G[tag + "_snd"], G[tag + "_rcv"], G[tag + "_r"], G[tag + "_diff"])
    assert got[2].ndim == 1


def test_nodes_within_radius_matches_reference():
    v = gu._nodes_within_radius(float(G["within_rad"]), G["within_pos1"], G["within_pos2"])
    assert v.shape == (len(G["within_pos2"]), 1)
    np.testing.assert_array_equal(v.ravel(), G["within_valid"])


@pytest.mark.parametrize("n1,n2", [(700, None), (130, 2100), (1, 65), (64, 64)])
def test_larger_and_ragged_sizes_vs_oracle(n1, n2):
    """Rows longer than a wave (several 64-column sweeps), ragged tails, one row."""
    rs = np.random.RandomState(n1)
    p1 = rs.uniform(0, 20, size=(n1, 2))
    p2 = None if n2 is None else rs.uniform(0, 20, size=(n2, 2))
    for self_loops in (False, True):
        s, q, r, d = og.radius_edges(1.5, p1, p2, self_loops)
        same(gu._get_graph_edges(1.5, p1, p2, self_loops), s, q, r, d.reshape(-1, 2))
        for k, near in ((1, True), (4, False), (9, True)):
            s, q, r, d = og.k_edges(k, p1, p2, self_loops, near)
            same(gu._get_k_edges(k, p1, p2, self_loops, near), s, q, r, d)


def test_ties_nan_coincident_and_errors():
    """Grid points (equal distances at the k-th boundary: lower column first, the
    oracle's rule), coincident points (r = 0 is not a radius edge), a NaN point (a NaN
    distance is a radius edge; np.argmin's first-NaN rule in _get_k_edges), empty input
    and kth out of bounds."""
    xs, ys = np.meshgrid(np.arange(7) * 5.5, np.arange(5) * 5.5)
    grid = np.stack([xs.ravel(), ys.ravel()], axis=1)
    for k, near in ((4, False), (3, True), (8, False)):
        s, q, r, d = og.k_edges(k, grid, None, False, near)
        same(gu._get_k_edges(k, grid, allow_nearest=near), s, q, r, d)
    pts = np.random.RandomState(2).uniform(0, 5, size=(50, 2))
    pts[7] = pts[3]
    pts[11] = np.nan
    for self_loops in (False, True):
        s, q, r, d = og.radius_edges(2.0, pts, None, self_loops)
        same(gu._get_graph_edges(2.0, pts, self_loops=self_loops), s, q, r, d.reshape(-1, 2))
    for near in (False, True):
        s, q, r, d = og.k_edges(3, pts, None, False, near)
        same(gu._get_k_edges(3, pts, allow_nearest=near), s, q, r, d)
    v = gu._nodes_within_radius(1.0, pts[:20], pts)
    np.testing.assert_array_equal(v.ravel(), og.nodes_within_radius(1.0, pts[:20], pts))
    (s, q), r, d = gu._get_graph_edges(1.0, np.zeros((0, 2)), pts)
    assert len(s) == len(q) == len(r) == 0 and d.shape == (0, 2)
    with pytest.raises(ValueError):
        gu._get_k_edges(5, pts[:5])
    with pytest.raises(ValueError):
        gu._get_k_edges(3, pts, np.zeros((3, 2)))
