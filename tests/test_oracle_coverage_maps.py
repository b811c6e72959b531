"""The restatement of the device map algorithm (oracle/coverage_maps.py) pinned on the
CPU: against the reference's recorded maps (tests/golden/coverage_maps.npz, made by
tests/golden/make_golden_coverage.py from /root/reference), against scipy's Delaunay
(the reference's make_map.py:213-219) on many city sets, against numpy's own
np.linalg.norm for the road lengths (make_map.py:227), and the library's host lattice
(cov_map_lattice, no device) against generate_lattice's recorded points."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import coverage_maps as cmo


def _fixture_maps():
    f = np.load(os.path.join(GOLDEN, "coverage_maps.npz"))
    lat, out, o = f["lattice"], [], 0
    for n in f["many_len"]:
        out.append(lat[f["many_idx"][o:o + n]])
        o += n
    return f, out


def test_restated_maps_match_reference_maps():
    """The first 30 recorded seeds (the GPU test runs all 100), and the second map of the
    first 4 streams."""
    f, many = _fixture_maps()
    for s in range(30):
        t, amb = cmo.generate_targets(cmo.cities(np.random.RandomState(s)))
        assert not amb
        np.testing.assert_array_equal(t, many[s], err_msg="seed %d" % s)
    lat = f["lattice"]
    o = 0
    for s, n in enumerate(f["next_len"][:4]):
        rs = np.random.RandomState(s)
        cmo.cities(rs)
        t, _ = cmo.generate_targets(cmo.cities(rs))
        np.testing.assert_array_equal(t, lat[f["next_idx"][o:o + n]])
        o += n


def test_cities_are_numpy_uniform():
    for s in (0, 7, 2**31 + 5):
        np.testing.assert_array_equal(cmo.cities(np.random.RandomState(s)),
                                      np.random.RandomState(s).uniform(-120, 120, size=(12, 2)))


def test_bruteforce_delaunay_equals_scipy():
    """The empty-circumcircle triangles' edges equal scipy's vertex_neighbor_vertices
    (Qhull) on 400 random city sets, none of them near-degenerate."""
    from scipy.spatial import Delaunay
    for s in range(400):
        c = cmo.cities(np.random.RandomState(50000 + s))
        ind, ptr = Delaunay(c).vertex_neighbor_vertices
        ref = sorted((i, int(j)) for i in range(len(c)) for j in ptr[ind[i]:ind[i + 1]] if i < j)
        got, amb = cmo.delaunay_edges(c)
        assert not amb
        assert got == ref, s


def test_cocircular_cities_are_reported():
    """Four cities on one circle (exactly cocircular in floating point: a square) are
    flagged instead of decided."""
    c = np.array([[0.0, 0.0], [10.0, 0.0], [10.0, 10.0], [0.0, 10.0], [30.0, 40.0], [-20.0, 35.0]])
    _, amb = cmo.delaunay_edges(c)
    assert amb


def test_road_length_is_numpy_norm():
    """np.linalg.norm of a (1, 2) difference is sqrt(x.dot(x)); the restatement's fused
    multiply-add form equals it on 20,000 city pairs (and differs from the unfused sum
    on some of them, so the form matters)."""
    rs = np.random.RandomState(3)
    differ = 0
    for _ in range(20000):
        p1, p2 = rs.uniform(-120, 120, size=(1, 2)), rs.uniform(-120, 120, size=(1, 2))
        d = p1 - p2
        ref = np.linalg.norm(d)
        assert cmo.road_length(p1[0], p2[0]) == ref
        differ += float(np.sqrt(d[0, 0] * d[0, 0] + d[0, 1] * d[0, 1])) != ref
    assert differ > 0


@pytest.mark.parametrize("arena", [(120, 120, 5.5), (57.3, 33, 5.5), (100, 80, 4.0), (120.5, 7.25, 5.5)])
def test_library_lattice_equals_generate_lattice(arena):
    """cov_map_lattice (the library's host code) against the restated generate_lattice,
    and at the reference's arena against its recorded lattice."""
    nat = pytest.importorskip("gym_flock._native")
    try:
        nat.load()
    except ImportError as e:
        pytest.skip(str(e))
    xm, ym, s = arena
    got = nat.map_lattice(nat.map_config_default(xmax=xm, ymax=ym, spacing=s))
    np.testing.assert_array_equal(got, cmo.lattice(-xm, xm, -ym, ym, s)[0])
    if arena == (120, 120, 5.5):
        np.testing.assert_array_equal(got, np.load(os.path.join(GOLDEN, "coverage_maps.npz"))["lattice"])
