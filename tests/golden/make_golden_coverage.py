"""Coverage-v0 golden vectors from the reference (imported by make_golden.py, which
installs the gym stub first). Records, per episode: the generated target graph, the
reset observation, and for a fixed action sequence every step's observation, reward,
done flag, robot nodes and visited set.

Config 4 of BASELINE.json needs non-default arguments (SURVEY.md finding 7):
n_robots=200, nearby_starts=False, max_nodes=1000.
"""
import importlib
import os

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))


def _episode(cov, n_robots, max_nodes, map_seed, env_seed, n_steps, policy, tag):
    np.random.seed(map_seed)  # the target graph is drawn from the global RNG
    env = cov.CoverageEnv(n_robots=n_robots, nearby_starts=False, max_nodes=max_nodes)
    env.seed(env_seed)
    np.random.seed(map_seed)  # reset() regenerates the same graph from the same draws
    obs = env.reset()
    R, T = env.n_robots, env.n_targets
    rec = dict(n_robots=R, n_targets=T, max_nodes=env.max_nodes,
               targets=env.x[R:, :2].copy(), motion_senders=np.array(env.motion_edges[0]),
               motion_receivers=np.array(env.motion_edges[1]),
               x0=env.x.copy(), visited0=env.visited[:, 0].copy(),
               nodes0=obs["nodes"].copy(), edges0=obs["edges"].copy(),
               senders0=np.array(obs["senders"]).copy(), receivers0=np.array(obs["receivers"]).copy(),
               step0=np.array(obs["step"]).copy())
    rs = np.random.RandomState(env_seed + 77)
    acts, xs, rews, dones, nodes, edges, snd, rcv, stp, vis, cls = ([] for _ in range(11))
    for t in range(n_steps):
        if policy == "random":
            a = rs.randint(0, 4, size=(R,))
        else:  # greedy expert (coverage.py:800-872, greedy branch); RNG only when stuck
            a = env.controller(random=False, greedy=True).flatten()
        acts.append(np.array(a).astype(np.int32))
        o, r, d, _ = env.step(np.array(a).reshape(-1, 1))
        xs.append(env.x[:R].copy()); rews.append(r); dones.append(d)
        nodes.append(o["nodes"].copy()); edges.append(o["edges"].copy())
        snd.append(np.array(o["senders"]).copy()); rcv.append(np.array(o["receivers"]).copy())
        stp.append(np.array(o["step"]).copy()); vis.append(env.visited[:, 0].copy())
        cls.append(np.array(env.closest_targets).astype(np.int32))
    if policy == "greedy":  # the reference's own time matrix (construct_time_matrix :621-653)
        rec.update(graph_cost=env.graph_cost.astype(np.int16), graph_previous=env.graph_previous.astype(np.int16))
    rec.update(actions=np.array(acts), xr=np.array(xs), reward=np.array(rews), done=np.array(dones),
               nodes=np.array(nodes, dtype=np.float32), edges=np.array(edges, dtype=np.float32),
               senders=np.array(snd, dtype=np.int32), receivers=np.array(rcv, dtype=np.int32),
               step=np.array(stp), visited=np.array(vis, dtype=np.int8), closest=np.array(cls))
    np.savez_compressed(os.path.join(OUT, "coverage_%s.npz" % tag), **rec)
    print("coverage %s: R=%d T=%d reward sum %d" % (tag, R, T, int(np.sum(rews))))


def gen_coverage():
    cov = importlib.import_module("gym_flock.envs.spatial.coverage")
    _episode(cov, 6, 500, map_seed=3, env_seed=4, n_steps=40, policy="random", tag="r6_random")
    _episode(cov, 6, 500, map_seed=5, env_seed=6, n_steps=30, policy="greedy", tag="r6_greedy")
    _episode(cov, 200, 1000, map_seed=8, env_seed=9, n_steps=12, policy="random", tag="r200_random")
    _episode(cov, 20, 700, map_seed=12, env_seed=13, n_steps=75, policy="greedy", tag="r20_greedy")
    gen_maps()


def gen_maps(n_seeds=100, n_next=10):
    """The map generator, pinned separately (coverage.py:516-527): seeds 0-2 as target
    arrays; seeds 0..n_seeds-1 as indices into the lattice (every target is a lattice
    point), and for seeds 0..n_next-1 the second map the same global stream draws (the
    next reset() after np.random.seed(s))."""
    cov = importlib.import_module("gym_flock.envs.spatial.coverage")
    mm = importlib.import_module("gym_flock.envs.spatial.make_map")
    lat = mm.generate_lattice((-120, 120, -120, 120), [np.array([-5.5, 0.]), np.array([0., -5.5])])
    where = {tuple(p): k for k, p in enumerate(lat.tolist())}
    env = cov.CoverageEnv(n_robots=6, nearby_starts=False, max_nodes=1000, init_graph=False)
    maps = {}
    many, nxt = [], []
    for s in range(n_seeds):
        np.random.seed(s)
        t, _ = env._generate_targets()
        if s < 3:
            maps["targets_seed%d" % s] = t
        many.append(np.array([where[tuple(p)] for p in t.tolist()], np.int16))
        if s < n_next:
            t2, _ = env._generate_targets()
            nxt.append(np.array([where[tuple(p)] for p in t2.tolist()], np.int16))
    np.savez_compressed(os.path.join(OUT, "coverage_maps.npz"), lattice=lat, **maps,
                        many_len=np.array([len(m) for m in many], np.int32), many_idx=np.concatenate(many),
                        next_len=np.array([len(m) for m in nxt], np.int32), next_idx=np.concatenate(nxt))
    print("coverage maps: %d seeds, %d targets on average" % (n_seeds, int(np.mean([len(m) for m in many]))))
