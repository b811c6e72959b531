"""Per-episode target maps for Coverage-v0 on the host, with scipy as the reference uses.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's CPU baseline, never by the
product (the product draws maps on the device, cov_generate_maps; oracle/coverage_maps.py
restates that device algorithm). Same algorithm and random draws as the reference's map
generation so a seeded global
NumPy RNG yields the reference's target set: a square lattice over the arena
(make_map.py:30-67), "roads" along the Delaunay edges of 12 random cities
(make_map.py:207-231), lattice points within motion_radius/1.4 of a road, and the
largest connected component of the motion graph (coverage.py:516-527).
"""
import numpy as np
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import connected_components
from scipy.spatial import Delaunay


def square_lattice(xmin, xmax, ymin, ymax, spacing):
    """make_map.generate_lattice with lattice vectors (-spacing, 0), (0, -spacing):
    returns (n, 2) points as [y, x] columns like the reference."""
    w, h = xmax - xmin, ymax - ymin
    nx, ny = w // spacing, h // spacing
    i = np.arange(-nx, nx, dtype=float)[:, None]
    j = np.arange(-ny, nx, dtype=float)[None, :]  # the reference's upper bound is nx here too
    px = -spacing * i + 0.0 * j
    py = 0.0 * i + -spacing * j
    keep = (px < w / 2.0) & (px > -w / 2.0) & (py < h / 2.0) & (py > -h / 2.0)
    px = px[keep] + (w // 2 + xmin)
    py = py[keep] + (h // 2 + ymin)
    return np.stack([py, px], axis=1)


def road_waypoints(n_cities, world_radius, road_radius, rng=np.random):
    """make_map.generate_geometric_roads: cities U(-r, r)^2, their Delaunay edges, and
    points every road_radius along each edge."""
    cities = rng.uniform(-world_radius, world_radius, size=(n_cities, 2))
    indptr_list, nbrs = Delaunay(cities).vertex_neighbor_vertices
    points = [cities]
    for a in range(cities.shape[0]):
        for b in nbrs[indptr_list[a]:indptr_list[a + 1]]:
            if a < b:
                p1, p2 = cities[a:a + 1], cities[b:b + 1]
                d = np.linalg.norm(p1 - p2)
                step = (p2 - p1) / d
                points.extend(p1 + step * k * road_radius for k in range(int(d / road_radius)))
    return np.vstack([points[0], np.vstack(points[1:])])


def _pairwise_sq(a, b):
    """Squared distances as np.linalg.norm(a[:, None] - b[None], axis=2) sums them before
    its sqrt (d0*d0 + d1*d1), without the (n, m, 2) temporaries."""
    dx = a[:, None, 0] - b[None, :, 0]
    dy = a[:, None, 1] - b[None, :, 1]
    return dx * dx + dy * dy


def generate_targets(xmax=120, ymax=120, res=5.5, motion_radius=None, n_cities=12, rng=np.random):
    """CoverageEnv._generate_targets (coverage.py:516-527)."""
    if motion_radius is None:
        motion_radius = res * 1.2
    lattice = square_lattice(-xmax, xmax, -ymax, ymax, res)
    roads = road_waypoints(n_cities, xmax, motion_radius, rng)
    # min over roads of the norms = sqrt of the min squared norm (sqrt is monotone and
    # correctly rounded), so one sqrt per lattice point decides the same set
    near = np.sqrt(np.min(_pairwise_sq(lattice, roads), axis=1)) <= (motion_radius / 1.4)
    targets = lattice[near, :]
    r = np.sqrt(_pairwise_sq(targets, targets))
    r[r > motion_radius] = 0
    _, labels = connected_components(csgraph=csr_matrix(r), directed=False, return_labels=True)
    return targets[labels == np.argmax(np.bincount(labels)), :]
