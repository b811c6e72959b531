"""Generate golden vectors from the gym-flock reference (run in the build container only).

This script is the ONLY place that executes reference code. It imports the
reference read-only from /root/reference through a minimal `gym` stand-in (the
reference imports `gym.Env`, `gym.spaces` and `gym.utils.seeding`, none of which
are installed here) and records inputs/outputs as small .npz fixtures under
tests/golden/. Nothing from the reference is copied: the fixtures are data
(states, actions and the reference's outputs for them).

Shim recipe: stub `gym`; numpy-2 aliases np.Inf/np.int/np.float;
bypass gym_flock/__init__.py (it calls gym.envs.registration.register) by
registering namespace packages whose __path__ points into the reference.

Usage:  python tests/golden/make_golden.py            (writes tests/golden/*.npz)
"""
import importlib
import os
import sys
import types

import numpy as np

REF = os.environ.get("GYMFLOCK_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------- shims
def _install_shims():
    import matplotlib
    matplotlib.use("Agg")
    import numpy.ma  # noqa: F401  (must import before aliasing)
    import scipy.sparse  # noqa: F401
    import scipy.spatial  # noqa: F401
    np.Inf = np.inf
    np.int = int
    np.float = float

    gym = types.ModuleType("gym")

    class Env:  # plain base class; the reference only subclasses it
        pass

    class _Space:
        def __init__(self, *args, **kwargs):
            self.args, self.kwargs = args, kwargs
            self.shape = kwargs.get("shape")

    spaces = types.ModuleType("gym.spaces")
    spaces.Box = type("Box", (_Space,), {})
    spaces.MultiDiscrete = type("MultiDiscrete", (_Space,), {})
    spaces.Dict = type("Dict", (_Space,), {})
    seeding = types.ModuleType("gym.utils.seeding")
    seeding.np_random = lambda seed=None: (np.random.RandomState(seed), seed)
    utils = types.ModuleType("gym.utils")
    utils.seeding = seeding
    error = types.ModuleType("gym.error")
    gym.Env, gym.spaces, gym.utils, gym.error = Env, spaces, utils, error
    sys.modules.update({"gym": gym, "gym.spaces": spaces, "gym.utils": utils,
                        "gym.utils.seeding": seeding, "gym.error": error})

    def ns(name, path):
        m = types.ModuleType(name)
        m.__path__ = [path]
        sys.modules[name] = m
        return m

    ns("gym_flock", os.path.join(REF, "gym_flock"))
    ns("gym_flock.envs", os.path.join(REF, "gym_flock", "envs"))
    ns("gym_flock.envs.flocking", os.path.join(REF, "gym_flock", "envs", "flocking"))
    ns("gym_flock.envs.spatial", os.path.join(REF, "gym_flock", "envs", "spatial"))


class _Cfg:
    """configparser-section stand-in exposing getfloat/getint (flocking_relative.py:68-85)."""

    def __init__(self, **kv):
        self.kv = kv

    def getfloat(self, k):
        return float(self.kv[k])

    def getint(self, k):
        return int(self.kv[k])


def synthetic_state(n, seed, v_max=5.0):
    """SURVEY §8d synthetic init: one draw of the reset() distribution, no rejection."""
    rs = np.random.RandomState(seed)
    r_max = np.sqrt(n)
    x = np.zeros((n, 4))
    length = np.sqrt(rs.uniform(0, r_max, size=(n,)))
    angle = np.pi * rs.uniform(0, 2, size=(n,))
    x[:, 0] = length * np.cos(angle)
    x[:, 1] = length * np.sin(angle)
    bias = rs.uniform(low=-v_max, high=v_max, size=(2,))
    x[:, 2] = rs.uniform(low=-v_max, high=v_max, size=(n,)) + bias[0]
    x[:, 3] = rs.uniform(low=-v_max, high=v_max, size=(n,)) + bias[1]
    return x


def make_flock_env(mod, n):
    env = mod.FlockingRelativeEnv()
    env.params_from_cfg(_Cfg(comm_radius=0.9, n_agents=n, v_max=5.0, dt=0.01))
    return env


def snapshot(env):
    adj = env.adj_mat > 0
    return dict(state_values=np.array(env.state_values), adj_bits=np.packbits(adj, axis=1),
                deg=adj.sum(axis=1).astype(np.int32))


# --------------------------------------------------------------------------- fixtures
def gen_flocking():
    fr = importlib.import_module("gym_flock.envs.flocking.flocking_relative")
    fl = importlib.import_module("gym_flock.envs.flocking.flocking")

    # (1) config 1: N=10 episode from the reference's own reset() (global np.random) with
    #     closed-loop expert actions (float64), then 20 steps with float32 random actions.
    n = 10
    np.random.seed(2024)
    env = make_flock_env(fr, n)
    sv0, net0 = env.reset()
    rec = dict(x0=env.x.copy(), sv0=sv0, net0=net0, r_max=env.r_max)
    xs, svs, nets, rews, us, ctrls = [], [], [], [], [], []
    for t in range(20):
        u = env.controller()
        us.append(u)
        (sv, net), r, done, _ = env.step(u)
        xs.append(env.x.copy()); svs.append(sv); nets.append(net); rews.append(r)
        ctrls.append(env.controller())
    rs = np.random.RandomState(7)
    for t in range(20):
        u = rs.uniform(-1, 1, size=(n, 2)).astype(np.float32)
        us.append(u.astype(np.float64))
        (sv, net), r, done, _ = env.step(u)
        xs.append(env.x.copy()); svs.append(sv); nets.append(net); rews.append(r)
        ctrls.append(env.controller())
    rec.update(u=np.array(us), u_is_f32=np.array([0] * 20 + [1] * 20, np.int8), x=np.array(xs),
               sv=np.array(svs), net=np.array(nets), reward=np.array(rews), ctrl=np.array(ctrls))
    np.savez_compressed(os.path.join(OUT, "flock_n10_episode.npz"), **rec)

    # (2) reset() at N=64 (rejection sampler, global RNG): pins our reset's RNG call order.
    np.random.seed(11)
    env = make_flock_env(fr, 64)
    env.reset()
    np.savez_compressed(os.path.join(OUT, "flock_n64_reset.npz"), seed=11, x0=env.x.copy(),
                        r_max=env.r_max, **snapshot(env))

    # (3) one step from a synthetic state, per (N, seed): float32 u and float64 u.
    for n, seeds in ((64, (1, 2)), (256, (3,)), (1024, (5, 6))):
        for seed in seeds:
            x0 = synthetic_state(n, seed)
            rs = np.random.RandomState(1000 + seed)
            u32 = rs.uniform(-1, 1, size=(n, 2)).astype(np.float32)
            rec = dict(x0=x0, u=u32)
            env = make_flock_env(fr, n)
            env.x = x0.copy()
            (sv, net), r, _, _ = env.step(u32)
            rec.update(x1=env.x.copy(), reward=r, **snapshot(env))
            rec["ctrl"] = env.controller()
            rec["ctrl_decentralized"] = env.controller(centralized=False)
            st = env.get_stats()
            rec["vel_diffs"], rec["min_dists"] = st["vel_diffs"], st["min_dists"]
            # Flocking-v0 observation on the same post-step state (flocking.py:20-25)
            kenv = fl.FlockingEnv()
            kenv.params_from_cfg(_Cfg(comm_radius=0.9, n_agents=n, v_max=5.0, dt=0.01))
            kenv.x = env.x.copy()
            kenv.compute_helpers()
            if n <= 256:  # at N=1024 the obs is implied by knn_idx and x1 (obs = x1[i] - x1[nn])
                rec["knn_obs"] = kenv.get_observation()
            rec["knn_idx"] = np.argsort(kenv.r2, axis=1)[:, :7].astype(np.int32)
            # float64 actions (what controller() returns) from the same start state
            u64 = rs.uniform(-1, 1, size=(n, 2))
            env.x = x0.copy()
            (sv64, _), r64, _, _ = env.step(u64)
            rec.update(u64=u64, x1_u64=env.x.copy(), sv_u64=sv64, reward_u64=r64,
                       deg_u64=(env.adj_mat > 0).sum(axis=1).astype(np.int32))
            np.savez_compressed(os.path.join(OUT, "flock_n%d_s%d_step.npz" % (n, seed)), **rec)
            print("flock N=%d seed=%d: reward %.6f mean deg %.2f" % (n, seed, r, rec["deg"].mean()))


if __name__ == "__main__":
    _install_shims()
    if "--only-extra" not in sys.argv:
        gen_flocking()
    if "--variants" in sys.argv or "--all" in sys.argv:
        from make_golden_variants import gen_variants  # noqa: E402
        gen_variants()
    if "--coverage" in sys.argv or "--all" in sys.argv:
        from make_golden_coverage import gen_coverage  # noqa: E402
        gen_coverage()
    elif "--maps" in sys.argv:
        from make_golden_coverage import gen_maps  # noqa: E402
        gen_maps()
    if "--graph-utils" in sys.argv or "--all" in sys.argv:
        from make_golden_graph_utils import gen_graph_utils  # noqa: E402
        gen_graph_utils()
