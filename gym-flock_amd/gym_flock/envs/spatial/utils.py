"""Graph helpers of gym_flock/envs/spatial/utils.py on the MI355X.

Same names, arguments and return values as the reference module:
`_get_graph_edges` (:8-24), `_nodes_within_radius` (:27-39), `_get_pos_diff` (:42-57)
and `_get_k_edges` (:60-88). The distance matrix, the radius / k-nearest selection and
the edge lists run in libgymflock.so (gu_* C-ABI, csrc/graph_utils.hip) on the device
named by GYMFLOCK_DEVICE (default 0); `_get_pos_diff` is the reference's broadcast
subtraction, returned as the ndarray callers index into.

Edges are returned like np.nonzero (a tuple of int64 arrays, row-major order), the
distances as float64, and the differences with the reference's layout: every edge's dx
followed by every dy (np.hstack), reshaped to (-1, 2) by _get_graph_edges and left 1-D
by _get_k_edges. Positions are taken as float64 (n, 2), which is what every reference
call site passes (coverage.py's x). Among EQUAL distances at the k-th boundary,
_get_k_edges keeps the lower column; numpy leaves that choice to its selection
algorithm.
"""
import os
import threading

import numpy as np

from ... import _native as nat

_local = threading.local()


def _graph():
    g = getattr(_local, "graph", None)
    if g is None:
        g = _local.graph = nat.GraphUtils(device=int(os.environ.get("GYMFLOCK_DEVICE", "0")))
    return g


def _edges(snd, rcv):
    return snd.astype(np.intp), rcv.astype(np.intp)


def _get_graph_edges(rad, pos1, pos2=None, self_loops=False):
    """utils.py:8-24: pairs with 0 != r and not r > rad -> (edges, r[edges], diff (E, 2))."""
    snd, rcv, r, diff = _graph().radius_edges(rad, pos1, pos2, self_loops)
    return _edges(snd, rcv), r, diff.reshape((-1, 2))


def _nodes_within_radius(rad, pos1, pos2):
    """utils.py:27-39: (n2, 1) bool, nodes of pos2 within rad of some point of pos1."""
    return _graph().nodes_within_radius(rad, pos1, pos2).reshape((-1, 1))


def _get_pos_diff(sender_loc, receiver_loc=None):
    """utils.py:42-57: diff[i, j] = sender_loc[i] - receiver_loc[j] (sender_loc if None)."""
    n, m = sender_loc.shape
    if receiver_loc is not None:
        n2, m2 = receiver_loc.shape
        return sender_loc.reshape((n, 1, m)) - receiver_loc.reshape((1, n2, m2))
    return sender_loc.reshape((n, 1, m)) - sender_loc.reshape((1, n, m))


def _get_k_edges(k, pos1, pos2=None, self_loops=False, allow_nearest=False):
    """utils.py:60-88: k outgoing edges per point of pos1 (the k nearest, or the k+1
    nearest minus the nearest) -> (edges, r[edges], diff (2E,)). Raises ValueError where
    the reference's np.argpartition does (kth >= len(pos2))."""
    try:
        snd, rcv, r, diff = _graph().k_edges(k, pos1, pos2, self_loops, allow_nearest)
    except nat.GymFlockError as e:
        if e.code == nat.GF_EINVAL:
            raise ValueError(str(e)) from None
        raise
    return _edges(snd, rcv), r, diff
