"""The graph-helper oracle (oracle/graph_utils.py) against the reference's recorded
outputs (tests/golden/graph_utils.npz): utils.py _get_graph_edges, _get_k_edges and
_nodes_within_radius. CPU only."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import graph_utils as gu

G = np.load(os.path.join(GOLDEN, "graph_utils.npz"))
RADIUS = sorted({k[:-5] for k in G.files if k.startswith("radius_") and k.endswith("_pos1")})
KNN = sorted({k[:-5] for k in G.files if k.startswith("k_") and k.endswith("_pos1")})


@pytest.mark.parametrize("tag", RADIUS)
def test_radius_edges_match_reference(tag):
    p2 = G[tag + "_pos2"] if tag + "_pos2" in G.files else None
    s, q, r, diff = gu.radius_edges(float(G[tag + "_rad"]), G[tag + "_pos1"], p2, bool(G[tag + "_self"]))
    np.testing.assert_array_equal(s, G[tag + "_snd"])
    np.testing.assert_array_equal(q, G[tag + "_rcv"])
    np.testing.assert_array_equal(r, G[tag + "_r"])
    np.testing.assert_array_equal(diff.reshape(-1, 2), G[tag + "_diff"])


@pytest.mark.parametrize("tag", KNN)
def test_k_edges_match_reference(tag):
    p2 = G[tag + "_pos2"] if tag + "_pos2" in G.files else None
    args = (int(G[tag + "_k"]), G[tag + "_pos1"], p2, bool(G[tag + "_self"]), bool(G[tag + "_near"]))
    assert gu.boundary_unique(*args)  # the recorded selection is unique
    s, q, r, diff = gu.k_edges(*args)
    np.testing.assert_array_equal(s, G[tag + "_snd"])
    np.testing.assert_array_equal(q, G[tag + "_rcv"])
    np.testing.assert_array_equal(r, G[tag + "_r"])
    np.testing.assert_array_equal(diff, G[tag + "_diff"])


def test_nodes_within_radius_matches_reference():
    v = gu.nodes_within_radius(float(G["within_rad"]), G["within_pos1"], G["within_pos2"])
    np.testing.assert_array_equal(v, G["within_valid"])


def test_k_edges_kth_out_of_bounds_raises():
    p = np.random.RandomState(0).uniform(size=(5, 2))
    with pytest.raises(ValueError):
        gu.k_edges(5, p)
    gu.k_edges(4, p)  # kth = 4 < 5 (the diagonal, +inf, is picked)
