"""CPU-side checks of the boundary: the C-ABI library loads and exports every symbol
include/gymflock.h declares, argument validation happens before any device work,
and the host-side Python logic (spaces, params_from_cfg, init states, sharding)
behaves like the reference. No kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gymflock.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+((?:fe|cov|gu)_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    for s in ("fe_create", "fe_step", "fe_controller", "fe_get_network", "fe_allgather_rewards",
              "cov_create", "cov_step", "cov_reset", "cov_get_obs", "gu_radius_edges", "gu_k_edges"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from gym_flock import _native as nat
    lib = nat.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
        assert s in nat.SIGNATURES, "binding missing for %s" % s
    assert lib.fe_abi_version() == 1


def test_create_validates_arguments_before_touching_the_device():
    from gym_flock import _native as nat
    lib = nat.load()
    h = ctypes.c_void_p()
    bad = [nat.FeConfig(0, 1, 0.9, 0.01, 10.0, 1, 1, 0, 0),      # n_agents 0
           nat.FeConfig(10, 0, 0.9, 0.01, 10.0, 1, 1, 0, 0),     # n_envs 0
           nat.FeConfig(5, 1, 0.9, 0.01, 10.0, 1, 1, 7, 0),      # k > N (reference IndexError)
           nat.FeConfig(50, 1, 0.9, 0.01, 10.0, 1, 1, 9, 0),     # unsupported k
           nat.FeConfig(10, 1, -1.0, 0.01, 10.0, 1, 1, 0, 0)]    # bad radius
    for cfg in bad:
        assert lib.fe_create(ctypes.byref(cfg), ctypes.byref(h)) == nat.GF_EINVAL
        assert lib.fe_last_error()
    assert lib.fe_step(None, None, 0) == nat.GF_EINVAL
    assert lib.fe_get_rewards(None, None) == nat.GF_EINVAL


def test_no_device_fails_loudly():
    """Without a GPU the product raises; there is no CPU fallback."""
    from gym_flock import _native as nat
    try:
        h = nat.FlockHandle(10, 1)
    except nat.GymFlockError as e:
        assert e.code == nat.GF_EHIP
        return
    h.close()
    pytest.skip("a GPU is present")


def test_step_shape_assertion_matches_reference():
    """flocking_relative.py:94 asserts u.shape == (n_agents, nu) before any work."""
    import gym_flock
    env = gym_flock.make("FlockingRelative-v0")
    with pytest.raises(AssertionError):
        env.step(np.zeros((99, 2)))
    with pytest.raises(AssertionError):
        env.step(np.zeros(200))


def test_params_from_cfg_matches_reference_semantics():
    import gym_flock

    class Cfg:
        def getfloat(self, k):
            return {"comm_radius": 1.2, "v_max": 3.0, "dt": 0.05}[k]

        def getint(self, k):
            return 16

    env = gym_flock.make("FlockingRelative-v0")
    env.params_from_cfg(Cfg())
    assert env.n_agents == 16 and env.comm_radius == 1.2 and env.dt == 0.05
    assert env.v_max == 3.0 and env.v_bias == 3.0
    assert env.r_max == pytest.approx(4.0)
    assert env.comm_radius2 == pytest.approx(1.44)
    assert env.action_space.shape == (32,) and env.observation_space.shape == (16, 6)
    env.params_from_cfg(Cfg())  # the reference compounds r_max (:75)
    assert env.r_max == pytest.approx(16.0)
    assert env.seed(3) == [3]


def test_host_init_states_match_oracle():
    from gym_flock.init_states import draw_swarm, synthetic_batch, synthetic_state
    from oracle import flocking as orc
    for n, s in ((10, 0), (1024, 5)):
        np.testing.assert_array_equal(synthetic_state(n, s), orc.synthetic_state(n, s))
    xb = synthetic_batch(3, 64, seed0=4)
    for b in range(3):
        np.testing.assert_array_equal(xb[b], orc.synthetic_state(64, 4 + b))
    # draw order of reset() with the global RNG: first candidate equals the oracle's
    np.random.seed(5)
    a = draw_swarm(20, np.sqrt(20), 5.0, 5.0)
    np.random.seed(5)
    rs = np.random.RandomState(5)
    b = draw_swarm(20, np.sqrt(20), 5.0, 5.0, rs)
    np.testing.assert_array_equal(a, b)


def test_golden_reset_fixture_is_reproduced_by_host_draws():
    """Replaying draw_swarm with the reference's acceptance test (evaluated by the
    oracle here) from the fixture's seed yields the reference's reset() state."""
    from conftest import GOLDEN
    from gym_flock.init_states import draw_swarm
    from oracle import flocking as orc
    f = np.load(os.path.join(GOLDEN, "flock_n64_reset.npz"))
    np.random.seed(int(f["seed"]))
    while True:
        x = draw_swarm(64, float(f["r_max"]), 5.0, 5.0)
        st = orc.stats(x)
        _, _, adj, deg = orc.helpers(x)
        if deg.min() >= 2 and st["min_dists"].min() >= 0.1:
            break
    np.testing.assert_array_equal(x, f["x0"])


def test_shard_range_partitions_the_batch():
    from gym_flock.shard import shard_range
    for total, world in ((2048, 8), (10, 3), (5, 8)):
        ranges = [shard_range(total, world, r) for r in range(world)]
        assert ranges[0][0] == 0 and ranges[-1][1] == total
        assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
        sizes = [b - a for a, b in ranges]
        assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_coverage_map_generation_matches_reference():
    """Host map generation (maps.py) reproduces the reference's target sets from the same
    global seeds (coverage.py:516-527, make_map.py:30-67, :207-231)."""
    from conftest import GOLDEN
    from oracle.maps_host import generate_targets, square_lattice
    f = np.load(os.path.join(GOLDEN, "coverage_maps.npz"))
    np.testing.assert_array_equal(square_lattice(-120, 120, -120, 120, 5.5), f["lattice"])
    for s in (0, 1, 2):
        np.random.seed(s)
        np.testing.assert_array_equal(generate_targets(), f["targets_seed%d" % s])
    for path in ("coverage_r6_random.npz", "coverage_r6_greedy.npz", "coverage_r200_random.npz"):
        g = np.load(os.path.join(GOLDEN, path))
        np.random.seed({"coverage_r6_random.npz": 3, "coverage_r6_greedy.npz": 5,
                        "coverage_r200_random.npz": 8}[path])
        np.testing.assert_array_equal(generate_targets(), g["targets"])


def test_coverage_create_validates_arguments():
    from gym_flock import _native as nat
    lib = nat.load()
    h = ctypes.c_void_p()
    for cfg in (nat.CovConfig(0, 1, 500, 75, 5.5, 6.6, 0), nat.CovConfig(6, 1, 6, 75, 5.5, 6.6, 0),
                nat.CovConfig(6, 0, 500, 75, 5.5, 6.6, 0), nat.CovConfig(6, 1, 500, 75, -1.0, 6.6, 0)):
        assert lib.cov_create(ctypes.byref(cfg), ctypes.byref(h)) == nat.GF_EINVAL


def test_reference_module_paths_import():
    """Callers import envs and helpers by the reference's module paths."""
    import importlib
    from gym_flock.envs.flocking import variants
    for mod, cls in (("flocking_leader", "FlockingLeaderEnv"), ("flocking_obstacle", "FlockingObstacleEnv"),
                     ("flocking_stoch", "FlockingStochasticEnv"), ("flocking_twoflocks", "FlockingTwoFlocksEnv")):
        m = importlib.import_module("gym_flock.envs.flocking." + mod)
        assert getattr(m, cls) is getattr(variants, cls)
    u = importlib.import_module("gym_flock.envs.spatial.utils")
    for fn in ("_get_graph_edges", "_get_k_edges", "_get_pos_diff", "_nodes_within_radius"):
        assert callable(getattr(u, fn))
    p = np.arange(6.0).reshape(3, 2)
    assert u._get_pos_diff(p).shape == (3, 3, 2) and u._get_pos_diff(p, p[:2]).shape == (3, 2, 2)


def test_shard_size_rule():
    """fe_comm_init all-gathers every rank's n_envs and applies fe_check_shard_sizes:
    uneven shards are accepted (the gathers pad every block to the largest shard);
    a size below 1 (a corrupted exchange: a handle always holds an env) is GF_ECOMM.
    The rule itself runs on the host."""
    from gym_flock import _native as nat
    nat.check_shard_sizes([256] * 8)
    nat.check_shard_sizes([3])
    nat.check_shard_sizes([256, 255])
    nat.check_shard_sizes([1, 2, 3, 4, 5, 6, 7, 8])
    for bad in ([4, 4, 4, 0], [2, -1]):
        with pytest.raises(nat.GymFlockError) as e:
            nat.check_shard_sizes(bad)
        assert e.value.code == nat.GF_ECOMM
        assert "bad env shard sizes" in str(e.value)


def test_unpad_gathered_layout():
    """shard.unpad_gathered on the RCCL gathers' block layout (rank-major blocks padded
    to the largest shard, include/gymflock.h): rewards (world, steps, W) and stats
    (world, W, 2) come back in global env order, padding dropped."""
    from gym_flock.shard import pad_block, shard_range, unpad_gathered
    total, world, steps = 11, 4, 3
    sizes = [b - a for a, b in (shard_range(total, world, r) for r in range(world))]
    W = max(sizes)
    rew = np.arange(steps * total, dtype=np.float64).reshape(steps, total) + 0.5
    st = np.arange(total * 2, dtype=np.float64).reshape(total, 2) - 7.25
    rblocks, sblocks = [], []
    for r in range(world):
        a, b = shard_range(total, world, r)
        rblocks.append(pad_block(rew[:, a:b], W, axis=1))
        sblocks.append(pad_block(st[a:b], W, axis=0))
    assert all(blk.shape == (steps, W) for blk in rblocks)
    np.testing.assert_array_equal(unpad_gathered(np.stack(rblocks), sizes, axis=1), rew)
    np.testing.assert_array_equal(unpad_gathered(np.stack(sblocks), sizes, axis=0), st)



def test_runtime_info_names_the_bound_libraries():
    """fe_runtime_info works without a device: the HIP runtime and RCCL versions and the
    shared objects libgymflock's HIP / RCCL entry points resolved to (this process has
    not loaded torch, so they are /opt/rocm's)."""
    from gym_flock import _native as nat
    info = nat.runtime_info()
    assert info["hip_runtime"] > 0 and info["rccl"] > 0, info
    assert "libamdhip64" in info["hip_lib"] and "librccl" in info["rccl_lib"], info
    assert os.path.exists(info["hip_lib"]) and os.path.exists(info["rccl_lib"]), info


def test_u_is_f64_follows_numpy_promotion():
    """float32 (and float16, computed as float32: its float16 rounding is unpinned) keep
    the float32 action arithmetic; float64 and integer arrays take float64, as NumPy's
    u * 10.0 promotes them (flocking_relative.py:95)."""
    from gym_flock import _native as nat
    assert not nat.u_is_f64(np.zeros(2, np.float32))
    assert not nat.u_is_f64(np.zeros(2, np.float16))
    assert (np.zeros(2, np.float16) * 10.0).dtype == np.float16  # NumPy itself stays in float16
    assert nat.u_is_f64(np.zeros(2, np.float64))
    assert nat.u_is_f64(np.zeros(2, np.int64))
