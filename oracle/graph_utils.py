"""CPU oracle for the graph helpers of gym_flock/envs/spatial/utils.py (SURVEY.md §8a
row a14).

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of the gu_* device
helpers; never by the product. Pinned against tests/golden/graph_utils.npz, recorded
from the reference (tests/golden/make_golden_graph_utils.py).

The k-nearest rows pick by (r, column) with NaN above +inf. np.argpartition leaves the
choice among equal distances at the k-th boundary to its selection algorithm, so that
choice is parity-unpinned; every recorded case has a unique boundary.
"""
import numpy as np


def pos_diff(p1, p2=None):
    """_get_pos_diff, utils.py:42-57: diff[i, j] = p1[i] - p2[j] (p2 = p1 if None)."""
    q = p1 if p2 is None else p2
    return p1[:, None, :] - q[None, :, :]


def dist(p1, p2=None):
    """np.linalg.norm(diff, axis=2) for 2-D points: sqrt(dx*dx + dy*dy)."""
    d = pos_diff(p1, p2)
    return np.sqrt(d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]), d


def radius_edges(rad, p1, p2=None, self_loops=False):
    """_get_graph_edges, utils.py:8-24: r > rad zeroed, the diagonal zeroed without self
    loops (pos2=None), edges = nonzero(r); diff = hstack(dx[edges], dy[edges])."""
    r, d = dist(p1, p2)
    r[r > rad] = 0
    if not self_loops and p2 is None:
        np.fill_diagonal(r, 0)
    s, q = np.nonzero(r)
    return s, q, r[s, q], np.hstack((d[s, q, 0], d[s, q, 1]))


def k_edges(k, p1, p2=None, self_loops=False, allow_nearest=False):
    """_get_k_edges, utils.py:60-88: the diagonal is +inf without self loops; per row the
    k smallest (allow_nearest) or the k+1 smallest with the row's argmin removed; edges
    in row-major order. Ties at the boundary: lower column first."""
    r, d = dist(p1, p2)
    if not self_loops and p2 is None:
        np.fill_diagonal(r, np.inf)
    n2 = r.shape[1]
    kth = k - 1 if allow_nearest else k
    if kth >= n2:
        raise ValueError("kth(=%d) out of bounds (%d)" % (kth, n2))
    key = np.where(np.isnan(r), np.inf, r)
    nan = np.isnan(r)
    mask = np.zeros(r.shape, bool)
    for i in range(r.shape[0]):
        order = np.lexsort((np.arange(n2), key[i], nan[i]))  # NaN last, then r, then column
        mask[i, order[:kth + 1]] = True
        if not allow_nearest:
            mask[i, np.argmin(r[i])] = False
    s, q = np.nonzero(mask)
    return s, q, r[s, q], np.hstack((d[s, q, 0], d[s, q, 1]))


def nodes_within_radius(rad, p1, p2):
    """_nodes_within_radius, utils.py:27-39: column sums of r (r > rad zeroed) > 0."""
    r, _ = dist(p1, p2)
    r[r > rad] = 0
    return np.sum(r, axis=0) > 0


def boundary_unique(k, p1, p2=None, self_loops=False, allow_nearest=False):
    """True when every row's (kth)-th and (kth+1)-th smallest distances differ, so the
    reference's selection is unique."""
    r, _ = dist(p1, p2)
    if not self_loops and p2 is None:
        np.fill_diagonal(r, np.inf)
    kth = k - 1 if allow_nearest else k
    srt = np.sort(r, axis=1)
    if kth + 1 >= r.shape[1]:
        return True
    return bool(np.all(srt[:, kth] != srt[:, kth + 1]))
