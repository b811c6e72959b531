"""CPU restatement of Coverage-v0's per-episode map generation, as the device does it.

TEST INFRASTRUCTURE ONLY: imported by tests/ (never by the product). Restates
CoverageEnv._generate_targets (gym_flock/envs/spatial/coverage.py:516-527) with its
helpers generate_lattice (make_map.py:30-67) and generate_geometric_roads
(make_map.py:207-231) in the form the device kernels use (coverage_maps.hip):

* the 12 cities: np.random.uniform(-r, r, (12, 2)) = -r + (r - -r) * random_sample
  (numpy's legacy uniform, make_map.py:208);
* the Delaunay edges of the cities (scipy.spatial.Delaunay, a Qhull wrapper absent from
  the device) as the union of the edges of every triangle whose circumcircle holds no
  other city strictly inside: the unique Delaunay triangulation of points in general
  position, which is what Qhull returns for them. Near-cocircular city sets (an incircle
  determinant inside its rounding bound) are reported, not decided: Qhull's own
  precision handling decides those (parity unpinned, probability ~1e-12 per map);
* each road's length as np.linalg.norm(p1 - p2) computes it for a (1, 2) array: the
  square root of x.dot(x), which numpy's bundled OpenBLAS ddot evaluates with a fused
  multiply-add here (fma(dy, dy, dx * dx); checked against numpy in
  tests/test_oracle_coverage_maps.py);
* the waypoints p1 + (p2 - p1) / dist * k * road_radius, k < int(dist / road_radius);
  their order does not matter (only their minimum distance to a lattice point does);
* lattice points whose nearest waypoint is within motion_radius / 1.4 (the square root
  of the minimum squared norm: sqrt is monotone and correctly rounded);
* the radius graph of those points and its largest connected component, ties to the
  component whose lowest index is smallest (scipy's connected_components numbers the
  components in order of their lowest node, and argmax(bincount) takes the first).
"""
from fractions import Fraction

import numpy as np

DELTA = 5.5  # coverage.py:61, the lattice vectors (-DELTA, 0), (0, -DELTA) (:125-128)

_EPS = 2.0 ** -53
_ICC_BOUND = 4.0 * (10.0 + 96.0 * _EPS) * _EPS   # Shewchuk's iccerrboundA, x4 margin
_CCW_BOUND = 4.0 * (3.0 + 16.0 * _EPS) * _EPS    # ccwerrboundA, x4 margin


def _floordiv(a, b):
    """Python's float floor division (numpy floor_divide on float64)."""
    return float(a // b)


def lattice(xmin, xmax, ymin, ymax, spacing=DELTA):
    """make_map.generate_lattice with lattice vectors (-spacing, 0), (0, -spacing): the
    (n, 2) points as [y, x] columns in the reference's order, and each point's (i, j)
    indices into arange(-nx, nx) x arange(-ny, nx)."""
    w, h = xmax - xmin, ymax - ymin
    cx, cy = w // 2, h // 2
    nx, ny = _floordiv(w, spacing), _floordiv(h, spacing)
    xs = np.arange(-nx, nx, dtype=float)
    ys = np.arange(-ny, nx, dtype=float)
    gi, gj = np.meshgrid(np.arange(len(xs)), np.arange(len(ys)), indexing="ij")
    xl = -spacing * xs[:, None] + 0.0 * ys[None, :]
    yl = 0.0 * xs[:, None] + -spacing * ys[None, :]
    keep = (xl < w / 2.0) & (xl > -w / 2.0) & (yl < h / 2.0) & (yl > -h / 2.0)
    pts = np.stack([yl[keep] + (cy + ymin), xl[keep] + (cx + xmin)], axis=1)
    return pts, gi[keep], gj[keep]


def cities(rs, n_cities=12, world_radius=120.0):
    """np.random.uniform(-r, r, size=(n, 2)) from the RandomState rs (make_map.py:208)."""
    lo, hi = -float(world_radius), float(world_radius)
    return lo + (hi - lo) * rs.random_sample((n_cities, 2))


def _orient(a, b, c):
    l = (a[0] - c[0]) * (b[1] - c[1])
    r = (a[1] - c[1]) * (b[0] - c[0])
    return l - r, _CCW_BOUND * (abs(l) + abs(r))


def _incircle(a, b, c, d):
    adx, ady = a[0] - d[0], a[1] - d[1]
    bdx, bdy = b[0] - d[0], b[1] - d[1]
    cdx, cdy = c[0] - d[0], c[1] - d[1]
    bdxcdy, cdxbdy = bdx * cdy, cdx * bdy
    cdxady, adxcdy = cdx * ady, adx * cdy
    adxbdy, bdxady = adx * bdy, bdx * ady
    alift = adx * adx + ady * ady
    blift = bdx * bdx + bdy * bdy
    clift = cdx * cdx + cdy * cdy
    det = alift * (bdxcdy - cdxbdy) + blift * (cdxady - adxcdy) + clift * (adxbdy - bdxady)
    perm = ((abs(bdxcdy) + abs(cdxbdy)) * alift + (abs(cdxady) + abs(adxcdy)) * blift
            + (abs(adxbdy) + abs(bdxady)) * clift)
    return det, _ICC_BOUND * perm


def delaunay_edges(c):
    """Edges (i < j) of the empty-circumcircle triangles; (edges, near_degenerate)."""
    n = len(c)
    adj = np.zeros((n, n), bool)
    amb = False
    for i in range(n):
        for j in range(i + 1, n):
            for k in range(j + 1, n):
                o, ob = _orient(c[i], c[j], c[k])
                if abs(o) <= ob:
                    amb = True
                    continue
                a, b, cc = (c[i], c[j], c[k]) if o > 0 else (c[i], c[k], c[j])
                inside, unsure = False, False
                for m in range(n):
                    if m in (i, j, k):
                        continue
                    d, db = _incircle(a, b, cc, c[m])
                    if d > db:
                        inside = True
                        break
                    if abs(d) <= db:
                        unsure = True
                if not inside:
                    amb = amb or unsure
                    adj[i, j] = adj[j, i] = adj[i, k] = adj[k, i] = adj[j, k] = adj[k, j] = True
    return [(i, j) for i in range(n) for j in range(i + 1, n) if adj[i, j]], amb


def _fma(x, y, z):
    return float(Fraction(x) * Fraction(y) + Fraction(z))


def road_length(p1, p2):
    """np.linalg.norm(p1 - p2) of (1, 2) rows: sqrt(x.dot(x)), ddot with a fused
    multiply-add."""
    dx, dy = p1[0] - p2[0], p1[1] - p2[1]
    return float(np.sqrt(_fma(dy, dy, dx * dx)))


def waypoints(c, edges, road_radius):
    pts = [np.asarray(c, float)]
    for i, j in edges:
        p1, p2 = c[i], c[j]
        dist = road_length(p1, p2)
        step = (p2 - p1) / dist
        n = int(dist / road_radius)
        if n:
            k = np.arange(n, dtype=float)[:, None]
            pts.append(p1[None, :] + (step[None, :] * k) * road_radius)
    return np.vstack(pts)


def _components_largest(points, link):
    n = len(points)
    parent = list(range(n))

    def find(x):
        while parent[x] != x:
            x = parent[x]
        return x

    d = np.sqrt((points[:, None, 0] - points[None, :, 0]) ** 2 + (points[:, None, 1] - points[None, :, 1]) ** 2)
    ii, jj = np.nonzero((d > 0) & (d <= link))
    for i, j in zip(ii.tolist(), jj.tolist()):
        ri, rj = find(i), find(j)
        if ri != rj:
            parent[max(ri, rj)] = min(ri, rj)
    roots = np.array([find(i) for i in range(n)])
    counts = np.bincount(roots, minlength=n)
    best = int(np.argmax(counts))  # the root is the component's lowest index
    return roots == best


def generate_targets(c, xmax=120, ymax=120, motion_radius=5.5 * 1.2, spacing=DELTA):
    """The map the device builds from the cities c: (targets (T, 2), near_degenerate)."""
    lat, _, _ = lattice(-xmax, xmax, -ymax, ymax, spacing)
    edges, amb = delaunay_edges(np.asarray(c, float))
    roads = waypoints(np.asarray(c, float), edges, motion_radius)
    dx = lat[:, None, 0] - roads[None, :, 0]
    dy = lat[:, None, 1] - roads[None, :, 1]
    near = np.sqrt(np.min(dx * dx + dy * dy, axis=1)) <= motion_radius / 1.4
    t = lat[near]
    return t[_components_largest(t, motion_radius)], amb
