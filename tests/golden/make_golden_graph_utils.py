"""Golden vectors for the graph helpers of gym_flock/envs/spatial/utils.py (SURVEY.md
§8a row a14), generated from the reference. make_golden.py imports this module after
installing its gym stub (python tests/golden/make_golden.py --only-extra --graph-utils).

Cases (inputs and the reference's outputs, nothing else):
  radius_*   _get_graph_edges on random points (pos2=None and a second set), on the
             Coverage grid map (many exactly equal distances: ties do not matter for a
             radius graph), with and without self loops, and with coincident points
  k_*        _get_k_edges on random points, where no two distances in a row are equal,
             so np.argpartition's choice is unique (allow_nearest on and off, pos2 given)
  within     _nodes_within_radius on random points
"""
import importlib
import os

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))


def gen_graph_utils():
    u = importlib.import_module("gym_flock.envs.spatial.utils")
    rec = {}

    def radius(tag, rad, p1, p2=None, self_loops=False):
        (s, q), r, diff = u._get_graph_edges(rad, p1, p2, self_loops=self_loops)
        rec.update({tag + "_pos1": p1, tag + "_rad": np.float64(rad), tag + "_self": np.int8(self_loops),
                    tag + "_snd": s.astype(np.int32), tag + "_rcv": q.astype(np.int32), tag + "_r": r,
                    tag + "_diff": diff})
        if p2 is not None:
            rec[tag + "_pos2"] = p2

    def knn(tag, k, p1, p2=None, self_loops=False, allow_nearest=False):
        (s, q), r, diff = u._get_k_edges(k, p1, p2, self_loops=self_loops, allow_nearest=allow_nearest)
        rec.update({tag + "_pos1": p1, tag + "_k": np.int32(k), tag + "_self": np.int8(self_loops),
                    tag + "_near": np.int8(allow_nearest), tag + "_snd": s.astype(np.int32),
                    tag + "_rcv": q.astype(np.int32), tag + "_r": r, tag + "_diff": diff})
        if p2 is not None:
            rec[tag + "_pos2"] = p2

    rs = np.random.RandomState(11)
    a = rs.uniform(0, 10, size=(150, 2))
    b = rs.uniform(0, 10, size=(90, 2))
    radius("radius_self", 1.3, a)
    radius("radius_loops", 1.3, a, self_loops=True)
    radius("radius_two", 1.1, a, b)
    dup = a[:40].copy()
    dup[5] = dup[3]  # a coincident pair: r = 0 is not an edge
    radius("radius_dup", 2.0, dup)
    xs, ys = np.meshgrid(np.arange(12) * 5.5, np.arange(9) * 5.5)
    grid = np.stack([xs.ravel(), ys.ravel()], axis=1)
    radius("radius_grid", 5.5 * 1.01, grid, self_loops=True)
    radius("radius_grid_diag", 5.5 * 1.5, grid)
    knn("k_excl", 4, a)
    knn("k_near", 4, a, allow_nearest=True)
    knn("k_two", 3, a[:60], b)
    knn("k_two_near", 6, a[:60], b, allow_nearest=True)
    knn("k_loops", 5, b, self_loops=True)
    c = rs.uniform(0, 10, size=(30, 2))
    w = u._nodes_within_radius(1.7, c, a)
    rec.update({"within_pos1": c, "within_pos2": a, "within_rad": np.float64(1.7), "within_valid": w.ravel()})
    np.savez_compressed(os.path.join(OUT, "graph_utils.npz"), **rec)
    print("graph_utils.npz: %d arrays" % len(rec))
