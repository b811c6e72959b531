#!/usr/bin/env python
"""Throughput of the FlockingRelative-v0 env step on MI355X, in agent-steps/s.

One "step" = one batched FlockingRelativeEnv.step() over all of this GPU's envs
(dynamics + compute_helpers + instant_cost, reference flocking_relative.py:91-147),
with the dense (N,N) float32 network, (N,6) state_values and rewards left in HBM.
Workload (BASELINE.json configs[1]): N=1024 agents x 256 envs per GPU, synthetic
random-init swarms, float32 actions U(-1,1) resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py is its own launcher: the
parent (which makes no GPU call) checks N against the GPUs it can see, spawns N fresh
worker processes of itself with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT set, relays rank 0's JSON line and exits non-zero if any worker fails. Under
torchrun, WORLD_SIZE must equal --gpus. `--dry-host` runs the same spawn, rendezvous and
whole-vector reward check with the CPU oracle's rewards and never loads HIP (CPU tests).

At one GPU the same JSON line also carries the other single-GPU configs of
BASELINE.json as sub-objects: "coverage_config4" (Coverage-v0, R=200, 512 envs) and
"n8192_config5" (N=8192 x 32 envs), each with ms_per_step, roofline and cpu_baseline;
plus the step + fused controller, the packed-adjacency output and the Flocking-v0
(k-nearest observation) forms of config 2.

Multi-GPU: the env batch is sharded (256 envs per rank, weak scaling, no exchange on
the step path); per-env rewards are all-gathered with RCCL on a side stream every 8
steps (the metrics path), and every rank checks the whole gathered vector. The worker
never imports torch: torchrun only launches it, and the ranks meet over a plain TCP
host channel (gym_flock.hostgroup) for the RCCL unique id, barriers and the max over
ranks of the timed region.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-flock_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
# with one launch per step, HIP events bracket every TIMING_EVERY-th launch; with split
# steps (the default) one event pair brackets the whole timed region
TIMING_EVERY = 8
# (N, envs per GPU, GPUs) -> which BASELINE.json config the run is
CONFIG_TAG = {(1024, 256, 1): " (BASELINE.json configs[1])", (1024, 256, 8): " (BASELINE.json configs[2])",
              (8192, 32, 1): " (BASELINE.json configs[4])"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


REWARM_STEPS = 512  # multi-rank runs: steps (with gathers) between RCCL init and the timed loop


def clock_warmup(step, sync, ms):
    """Steps until `ms` of wall time have passed, synchronising every 8 steps, so the
    GPU's clocks have left their idle state before anything is timed.

    Why (scripts/window_probe.py, profiles/r02/window_probe_v1.*): from a cold process
    consecutive 20-step windows of config 2 took 231, 216, 200, 190, 186, 183 us per
    step, i.e. the device reaches its sustained rate only after ~20 ms of load, and it
    drops back after idle gaps (1 s idle: 197 us; a host-side reset: 221 us). With the
    clocks warm the synthetic init state and a dispersed swarm step at the same rate
    (184 vs 186 us, scripts/init_probe.py). The caller restores the state afterwards, so
    the timed steps see the same inputs as without this warm-up; its length and step
    count are reported in the bench line ("clock_warmup")."""
    t0, n = time.perf_counter(), 0
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            step()
        sync()
        n += 8
    return {"ms": round(1e3 * (time.perf_counter() - t0), 1), "steps": n,
            "note": "untimed steps before the warmup steps (GPU clocks leave idle); the state is then "
                    "reset to the synthetic init, so the timed steps see the same inputs"}


def step_bytes(n):
    """Algorithmic HBM bytes of one env-step: read x (float64, 32N) +
    u (float32, 8N); write x (32N), state_values (float32, 24N), network (float32,
    4N^2) and the reward (8)."""
    return 4 * n * n + 96 * n + 8


def load_traffic(key):
    """Per-step HBM bytes measured by rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE, gfx950
    correction) for the workload `key` ("1024x256", "8192x32", "knn7_1024x256",
    "coverage_r200x512"), committed in profiles/pmc_traffic.json; None if absent."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(key)
        return None if e is None else float(e["bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


# ------------------------------------------------------------------ CPU baselines
def cpu_ref_rate(n_agents, seconds, seed=0, max_steps=100000):
    """oracle/cpu_ref.py: the reference's own NumPy array-op sequence for step()
    (checked bitwise and within 15 % of the reference's time by scripts/check_cpu_ref.py)
    on one env of the same synthetic workload, one thread."""
    from oracle.cpu_ref import CpuFlock
    from gym_flock.init_states import synthetic_state
    env = CpuFlock(synthetic_state(n_agents, seed))
    u = np.random.RandomState(1234 + seed).uniform(-1, 1, size=(n_agents, 2)).astype(np.float32)
    steps, t0 = 0, time.perf_counter()
    while True:
        env.step(u)
        steps += 1
        el = time.perf_counter() - t0
        if (el >= seconds and steps >= 1) or steps >= max_steps:
            return n_agents * steps / el, steps, el


def cpu_worker(n_agents, seconds, seed, pin_core=None):
    """--cpu-worker: one process of the CPU baseline (no GPU is touched), pinned to one
    core first when pin_core is given (sched_setaffinity, taskset's system call)."""
    if pin_core is not None:
        os.sched_setaffinity(0, {pin_core})
    rate, steps, el = cpu_ref_rate(n_agents, seconds, seed)
    print(json.dumps({"agent_steps_per_s": rate, "steps": steps, "seconds": el,
                      "affinity": sorted(os.sched_getaffinity(0))}), flush=True)


def cpu_workers(n_agents, seconds, cores, pin=True):
    """One single-threaded cpu_ref child process per entry of `cores`, all at once (OMP/BLAS
    threads 1), each pinned to its core when `pin`; returns their results."""
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-worker", str(seconds), "--n-agents", str(n_agents)]
    ps = [subprocess.Popen(cmd + ["--seed", str(k)] + (["--pin-core", str(c)] if pin else []),
                           stdout=subprocess.PIPE, env=env)
          for k, c in enumerate(cores)]
    res = []
    for p in ps:
        out, _ = p.communicate(timeout=seconds * 10 + 120)
        if p.returncode == 0:
            res.append(json.loads(out.decode().strip().splitlines()[-1]))
    return res


def flock_cpu_baseline(n_agents, seconds, procs=None):
    """the reference's op sequence (oracle/cpu_ref.py) on one core pinned
    (per_core), then on every core of the usable CPU share at once, one single-threaded
    process per core (value = the sum). The all-cores processes are not pinned: on the
    GPU box the cgroup grants a 16-CPU share of a 256-CPU host whose other tenants run on
    fixed cores; 16 processes pinned to the first 16 affinity cores measured 9.1e4 against
    2.6e5 left to the scheduler (profiles/r03)."""
    share = cpu_share()
    omp = os.environ.get("OMP_NUM_THREADS")
    use = procs or min(share["use"], int(omp) if omp and omp.isdigit() else share["use"])
    cores = share["cores"][:use] if use <= len(share["cores"]) else list(range(use))
    one = cpu_workers(n_agents, seconds, cores[:1])
    if not one:
        return {"value": None, "unit": "agent-steps/s", "error": "CPU baseline worker failed"}
    rate, steps, el = one[0]["agent_steps_per_s"], one[0]["steps"], one[0]["seconds"]
    out = {"value": rate, "unit": "agent-steps/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
           "per_core": rate, "nproc": share["nproc"], "affinity_cpus": share["affinity"],
           "cgroup_cpu_quota": share["cgroup_quota"], "omp_num_threads": omp,
           "sample": "oracle/cpu_ref.py step() on 1 env of N=%d for %d steps (%.1f s), 1 thread pinned to core %d: "
                     "the reference's own NumPy array-op sequence (flocking_relative.py:91-147), bitwise equal to it "
                     "and within 15%% of its time (scripts/check_cpu_ref.py, profiles/r03/cpu_ref_check.json); same "
                     "synthetic init and float32 actions as the GPU run" % (n_agents, steps, el, cores[0])}
    if use > 1:
        log("cpu baseline, all cores: %d processes x ~%.0fs..." % (use, seconds / 2))
        res = cpu_workers(n_agents, seconds / 2, cores, pin=False)
        out.update(value=sum(r["agent_steps_per_s"] for r in res), cores=len(res),
                   sample=out["sample"] + "; value = %d such processes at once (unpinned, within the cgroup's "
                                          "CPU share), one per CPU of the usable share (min of nproc=%d, "
                                          "affinity=%d, cgroup quota=%s, OMP_NUM_THREADS=%s), %.0f s, summed; "
                                          "per_core = one process alone, pinned"
                                          % (len(res), share["nproc"], share["affinity"], share["cgroup_quota"],
                                             omp, seconds / 2))
    return out


# ------------------------------------------------------------------ timed regions
class Ranks:
    """Barrier and max over ranks through the host channel (None: one process)."""

    def __init__(self, group):
        self.g = group

    def barrier(self, env):
        env.sync()
        if self.g is not None:
            self.g.barrier()

    def gather(self, v):
        """Every rank's value, in rank order."""
        return [float(v)] if self.g is None else self.g.allgather_f64(v)


def timed(env, ranks, k, step, per_rank=None):
    """k steps bracketed by a barrier + device sync on both sides; returns (max-over-
    ranks wall seconds, device ms per step from the handle's timing window). per_rank, if
    a list, receives every rank's wall seconds."""
    ranks.barrier(env)
    env.h.timing_start(every=TIMING_EVERY)
    t0 = time.perf_counter()
    for s in range(k):
        step(s)
    env.sync()
    el = time.perf_counter() - t0
    kernel_ms, _ = env.h.timing_stop()
    ranks.barrier(env)
    every = ranks.gather(el)
    if per_rank is not None:
        per_rank[:] = every
    return max(every), kernel_ms


def flock_roofline(n, b, kernel_ms, launches_per_step, kernel="flock_step_kernel<DYN,f32 u>"):
    bytes_step = b * step_bytes(n)
    achieved = bytes_step / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic("%dx%d" % (n, b)),
            "kernel": kernel, "region_ms_per_step": kernel_ms,
            "algorithmic_bytes_per_step": bytes_step, "launches_per_step": launches_per_step,
            "timing": "device time per step of the whole timed region (HIP events on the handle's stream, the "
                      "end event after it joins the second): each step is two concurrent half-batch launches "
                      "of the kernel on two streams, so region_ms_per_step and the bytes are per step"}


def bench_config5(args):
    """BASELINE.json configs[4]: N=8192 x 32 envs (the dense N^2 stress case)."""
    from gym_flock.vec import VecFlockingRelative
    # the headline's step count (each step is ~9x config 2's, so the window is long
    # enough that the last step's lagging half-launch does not weigh on it)
    N, B, K, W = 8192, 32, max(5, args.steps), max(2, args.warmup)
    env = VecFlockingRelative(B, N)
    x0 = env.reset(seed=0)
    env.set_actions(np.random.RandomState(1234).uniform(-1, 1, size=(B, N, 2)).astype(np.float32))
    warm = clock_warmup(lambda: env.step(resident=True), env.sync, 100.0)
    env.set_state(x0)
    for _ in range(W):
        env.step(resident=True)
    el, kms = timed(env, Ranks(None), K, lambda s: env.step(resident=True))
    env.close()
    out = {"metric": "agent-steps/sec, FlockingRelative N=8192", "value": N * B * K / el, "unit": "agent-steps/s",
           "steps": K, "warmup": W, "clock_warmup": warm, "ms_per_step": 1e3 * el / K,
           "config": {"workload": "FlockingRelative-v0 step(), N=8192 agents x 32 envs (BASELINE.json configs[4])"},
           "roofline": flock_roofline(N, B, kms, 2, kernel="flock_step_kernel<DYN,f32 u,PF> (tiles prefetched one ahead)")}
    if not args.no_cpu_baseline:
        log("cpu baseline N=8192 (cpu_ref, 1 step)...")
        rate, steps, sec = cpu_ref_rate(N, 1.0, max_steps=1)
        out["cpu_baseline"] = {"value": rate, "unit": "agent-steps/s", "cores": 1, "kind": "port",
                               "cpu_model": cpu_model(),
                               "sample": "oracle/cpu_ref.py step() (the reference's array-op sequence, ~12 GB of "
                                         "(N,N,{4,6}) float64 temporaries) on 1 env of N=8192 for %d step (%.1f s), "
                                         "1 thread" % (steps, sec)}
    return out


def coverage_cpu_baseline(targets, n_robots, max_nodes, seconds):
    """oracle/cpu_ref_coverage.py: the reference's own CoverageEnv.step op sequence
    (per-robot loops, np.where lookups, list-membership collision test, three R x T
    closest_targets argmins; coverage.py:174-364, :427-432), checked bitwise against the
    reference's recorded episodes (tests/test_oracle_coverage.py) and within 15 % of its
    time (scripts/check_cpu_ref.py), on one env of the same workload, one thread."""
    from oracle.cpu_ref_coverage import CpuCoverage
    rs = np.random.RandomState(0)
    env = CpuCoverage(targets, n_robots, max_nodes)
    T = len(targets)
    env.reset(rs.choice(T, n_robots, replace=False), rs.choice(T, T // 2, replace=False) + n_robots)
    acts = rs.randint(0, 4, size=(n_robots, 1))
    steps, t0 = 0, time.perf_counter()
    while True:
        env.step(acts)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds and steps >= 3:
            break
    return {"value": n_robots * steps / el, "unit": "robot-steps/s", "cores": 1, "kind": "port",
            "cpu_model": cpu_model(), "ms_per_env_step": 1e3 * el / steps,
            "sample": "oracle/cpu_ref_coverage.py step() (the reference's own loop/np.where op sequence, "
                      "coverage.py:174-364; bitwise equal to the reference's recorded episodes and within 15%% of "
                      "its time, profiles/r03/cpu_ref_check.json) on 1 env, R=%d, T=%d, %d steps (%.1f s), "
                      "1 thread" % (n_robots, T, steps, el)}


def bench_config4(args, with_greedy=False):
    """BASELINE.json configs[3]: Coverage-v0, 200 robots on a ~550-target map, 512 envs,
    max_nodes 1000 (the reference needs nearby_starts=False and max_nodes=1000 at this
    size, SURVEY.md finding 7). All envs share one generated map (global seed 8);
    starts, unvisited sets and actions differ per env; actions stay resident in HBM."""
    from oracle.maps_host import generate_targets
    from gym_flock.vec import VecCoverage
    # a Coverage step is ~9 us of latency-bound work: at least 1000 steps and 20 warm-up
    # steps per window, so neither the window's fixed start/end cost (~0.1 ms) nor the
    # first steps after the reset dominate (200-step windows after 5 warm-up steps read
    # 8.7-12.4 us on one build, profiles/r02/v5)
    R, B, M, K, W = 200, 512, 1000, max(1000, args.steps), max(20, args.warmup)
    np.random.seed(8)
    targets = generate_targets()
    v = VecCoverage(B, R, max_nodes=M, episode_length=10 ** 9)
    v.set_targets(targets)
    v.reset(seed=0)
    v.set_actions(np.random.RandomState(7).randint(0, 4, size=(B, R)))
    warm = clock_warmup(lambda: v.step(resident=True), v.sync, 100.0)
    v.reset(seed=0)  # the same starts and unvisited sets as without the warm-up
    for _ in range(W):
        v.step(resident=True)
    el, kernel_ms = timed(v, Ranks(None), K, lambda s: v.step(resident=True))
    # algorithmic bytes per env-step: the 8R-edge observation tail (sender, receiver,
    # edge: 12 B each) + per robot its action, node, position, visited flag and 4
    # action-target coordinates + the reward/done/step words
    per_env = 8 * R * 12 + R * (16 + 4 + 4 + 4 + 16) + 16
    achieved = B * per_env / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    out = {"metric": "robot-steps/sec (N_robots x N_envs x steps/s), Coverage-v0 R=200",
           "value": R * B * K / el, "unit": "robot-steps/s", "steps": K, "warmup": W, "clock_warmup": warm,
           "ms_per_step": 1e3 * el / K,
           "config": {"workload": "Coverage-v0 step(), R=200 robots, T=%d targets, max_nodes %d, %d envs "
                                  "(BASELINE.json configs[3])" % (len(targets), M, B)},
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic("coverage_r200x512"),
                        "kernel": "cov_step_kernel",
                        "region_ms_per_step": kernel_ms, "algorithmic_bytes_per_step": B * per_env,
                        "launches_per_step": 1,
                        "note": "latency-limited, not bandwidth-limited: one workgroup per env, two dependent "
                                "global round trips and the claim resolution per step (DESIGN.md); traffic from "
                                "PMC with the FETCH_SIZE x2 correction, which the guide calibrates for wide "
                                "coalesced reads only (these are scattered 4-64 B reads)"}}
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = coverage_cpu_baseline(targets, R, M, min(args.cpu_seconds, 8.0))
    if with_greedy:
        out["greedy_expert"] = bench_greedy(v, targets, R, M, B, K, args)
    v.close()
    out["distinct_maps"] = bench_config4_distinct_maps(args, R, B, M)
    return out


def bench_config4_distinct_maps(args, R, B, M, episodes=8):
    """Config 4 as the reference's reset() semantics imply: every env its own map (drawn on
    the device, cov_generate_maps, env b's stream seeded np.random.seed(8 + b)), episodes of
    the reference's EPISODE_LENGTH = 75 steps with random actions resident in HBM, each
    episode's reset (new starts and unvisited sets; the maps stay) outside the timed
    windows; then the same windows with one map shared by every env (the headline's
    workload) for the comparison. Also: a new map for all envs, timed."""
    from gym_flock.vec import VecCoverage
    rs = np.random.RandomState(7)

    def episodes_ms(v):
        v.reset(seed=0)
        v.set_actions(rs.randint(0, 4, size=(B, R)))
        clock_warmup(lambda: v.step(resident=True), v.sync, 50.0)
        el, k = 0.0, 0
        for e in range(episodes):
            v.reset(seed=1 + e)
            v.set_actions(rs.randint(0, 4, size=(B, R)))
            v.sync()
            t0 = time.perf_counter()
            for _ in range(75):
                v.step(resident=True)
            v.sync()
            el += time.perf_counter() - t0
            k += 75
        return 1e3 * el / k

    v = VecCoverage(B, R, max_nodes=M, episode_length=75)
    n, st = v.generate_maps(map_seed=8)
    v.sync()
    t0 = time.perf_counter()
    for _ in range(3):
        v.generate_maps()  # the next map of every stream: what each reference reset() draws
    map_ms = 1e3 * (time.perf_counter() - t0) / 3
    n, st = v.generate_maps(map_seed=8)
    distinct = episodes_ms(v)
    v.set_targets(v.h.targets(0, int(n[0])))  # env 0's map for every env
    shared = episodes_ms(v)
    v.close()
    return {"step_ms_distinct_maps": distinct, "step_ms_shared_map": shared,
            "robot_steps_per_s_distinct_maps": R * B / (distinct * 1e-3),
            "n_targets_min_mean_max": [int(n.min()), float(n.mean()), int(n.max())],
            "map_ms_all_envs": map_ms, "episodes": episodes,
            "note": "per step, %d episodes of 75 resident-action steps, resets untimed; distinct: env b's map from "
                    "np.random.seed(8 + b)'s stream; shared: env 0's map for all; map_ms_all_envs: one new map "
                    "for all %d envs (cities, Delaunay roads, lattice filter, largest component and the motion "
                    "graph, on the device)" % (episodes, B)}


def bench_dropin(args):
    """The drop-in single-env path existing GNN trainers call (flocking_relative.py:91-109,
    :194-212): FlockingRelativeEnv.step(u) with host actions in and host
    (state_values, network), reward out, one env per object, plus controller() each
    iteration (u = env.controller(); env.step(u), the expert loop). Per-call wall time at
    N=100 and N=1024 for each way of fetching the outputs ("getters": three synchronous
    getters; "batched": one fe_get_outputs call and one sync into fresh numpy arrays;
    "pooled": the same call into page-locked arrays from the env's HostPool; "direct", the
    env default: one fe_step_host call, the kernel reading the actions from and writing the
    outputs to page-locked memory, and computing the next expert action in the same launch
    once controller() is in use), with the reference's op sequence (oracle/cpu_ref.py)
    timed beside it on one core."""
    from gym_flock.envs.flocking.flocking_relative import FlockingRelativeEnv
    from gym_flock.init_states import synthetic_state
    from oracle.cpu_ref import CpuFlock
    out = {}
    for n, iters in ((100, 400), (1024, 100)):
        x0 = synthetic_state(n, 0)
        u32 = np.random.RandomState(5).uniform(-1, 1, size=(n, 2)).astype(np.float32)
        row = {}
        for mode in ("getters", "batched", "pooled", "direct"):
            env = FlockingRelativeEnv()
            env.n_agents = n
            env._make_spaces()
            env.fetch_mode = mode
            env.x = x0
            env.compute_helpers()

            def expert(k):
                for _ in range(k):
                    env.step(env.controller())

            def plain(k):
                for _ in range(k):
                    env.step(u32)

            r = {}
            for name, fn in (("step_ms", plain), ("controller_plus_step_ms", expert)):
                fn(20)
                t0 = time.perf_counter()
                fn(iters)
                r[name] = 1e3 * (time.perf_counter() - t0) / iters
            env.close()
            row[mode] = r
        cpu = CpuFlock(x0)
        k = 200 if n <= 100 else 3
        t0 = time.perf_counter()
        for _ in range(k):
            cpu.step(u32)
        t_step = (time.perf_counter() - t0) / k
        t0 = time.perf_counter()
        for _ in range(k):
            cpu.step(cpu.controller())
        t_ctrl = (time.perf_counter() - t0) / k
        row["cpu_ref_1core"] = {"step_ms": 1e3 * t_step, "controller_plus_step_ms": 1e3 * t_ctrl}
        # Flocking-v0's drop-in step (flocking.py:12-25): the observation is the 7-nearest
        # rows; "direct" (default) is one fe_step_host_knn call, "pooled" the older form
        from gym_flock.envs.flocking.flocking import FlockingEnv
        w = int(np.ceil(np.sqrt(n)))
        lattice = np.zeros((n, 4))  # an exact lattice at rest: every row's r2 tied, every step
        lattice[:, :2] = np.stack(np.meshgrid(np.arange(w), np.arange(w)), -1).reshape(-1, 2)[:n] * 0.5
        for mode in ("pooled", "direct"):
            env = FlockingEnv()
            env.n_agents = n
            env._make_spaces()
            env.fetch_mode = mode
            env.x = x0
            env.compute_helpers()

            def v0_plain(k):
                for _ in range(k):
                    env.step(u32)

            def v0_expert(k):
                for _ in range(k):
                    env.step(env.controller())

            r = {}
            for name, fn in (("step_ms", v0_plain), ("controller_plus_step_ms", v0_expert)):
                fn(20)
                t0 = time.perf_counter()
                fn(iters)
                r[name] = 1e3 * (time.perf_counter() - t0) / iters
            env.close()
            if mode == "direct":
                env = FlockingEnv()
                env.n_agents = n
                env._make_spaces()
                env.x = lattice
                env.compute_helpers()
                z = np.zeros((n, 2), np.float32)
                for _ in range(20):
                    env.step(z)
                t0 = time.perf_counter()
                for _ in range(iters):
                    env.step(z)
                r["lattice_at_rest_step_ms"] = 1e3 * (time.perf_counter() - t0) / iters
                env.close()
            row["flocking_v0_" + mode] = r
        out["n%d" % n] = row
    out["note"] = ("one env per FlockingRelativeEnv object, float32 host actions for step_ms, float64 controller() "
                   "output for controller_plus_step_ms; outputs copied to fresh host arrays every call, as the "
                   "reference returns them; the env default is fetch_mode='direct' (one launch and one wait per "
                   "step, the expert action of the new state fused into it); flocking_v0_*: FlockingEnv.step(u) (Flocking-v0, "
                   "7-nearest observation), 'direct' = one fe_step_host_knn(_ctrl) call (the expert action fused "
                   "once controller() is in use); lattice_at_rest: an exact lattice (spacing 0.5) with zero "
                   "velocities and actions, every row's r2 tied every step")
    return out


def bench_dropin_coverage(args):
    """The reference driver's loop (test.py:43-74) on one Coverage-v0 env through the
    drop-in API: `env.step(env.controller(random=True))` and `env.step(env.controller(
    greedy=True))`, whole episodes (reset every EPISODE_LENGTH steps or at done; resets
    untimed), per call, at R=6 (the module defaults: 500 padded nodes, nearby starts) and
    R=200 (max_nodes 1000, starts anywhere, as config 4). "direct" (the env default) is one
    cov_step_host call per step (the greedy actions of the next state fused into it);
    "getters" is cov_step then the observation and reward getters. The CPU side: the
    reference's own step op sequence (oracle/cpu_ref_coverage.py) with np.random choices,
    and with the greedy expert of oracle/coverage.py (a vectorised port, faster than the
    reference's controller) plus its time matrix per map."""
    from gym_flock.envs.spatial import CoverageEnv
    out = {}
    # max_nodes 1000 for both: the map generator's target count varies from reset to reset
    # (~390-560 here), and the module default of 500 padded nodes rejects the larger maps
    for R, M, nearby, episodes in ((6, 1000, True, 6), (200, 1000, False, 3)):
        row = {}
        for mode in ("getters", "direct"):
            for pol in ("random", "greedy"):
                np.random.seed(8)
                env = CoverageEnv(n_robots=R, nearby_starts=nearby, max_nodes=M)
                env.fetch_mode = mode
                env.seed(3)
                steps, el, first, el_first, el_reset = 0, 0.0, 0, 0.0, 0.0
                for ep in range(episodes + 1):  # the first episode warms up (not counted)
                    t0 = time.perf_counter()
                    env.reset()  # a new map (cities from np.random, the rest on the device)
                    if ep > 0:
                        el_reset += time.perf_counter() - t0
                    done, k = False, 0
                    while not done:
                        t0 = time.perf_counter()
                        a = env.controller(random=True) if pol == "random" else env.controller(greedy=True)
                        _, _, done, _ = env.step(a)
                        dt = time.perf_counter() - t0
                        if ep > 0:
                            steps += 1
                            el += dt
                            if k == 0:
                                first += 1
                                el_first += dt
                        k += 1
                env.close()
                r = {"step_ms": 1e3 * el / steps, "steps": steps, "reset_ms": 1e3 * el_reset / episodes,
                     "episode_ms_with_reset": 1e3 * (el + el_reset) / episodes}
                if pol == "greedy":  # the first step of an episode builds the new map's time matrix
                    r["step_ms_after_first"] = 1e3 * (el - el_first) / max(1, steps - first)
                    r["first_step_ms"] = 1e3 * el_first / max(1, first)
                row["%s_%s" % (mode, pol)] = r
        if not args.no_cpu_baseline:
            from oracle import coverage as oc
            from oracle.cpu_ref_coverage import CpuCoverage
            from oracle.maps_host import generate_targets
            np.random.seed(8)
            targets = generate_targets()
            T = len(targets)
            rs = np.random.RandomState(0)
            cpu = CpuCoverage(targets, R, M)
            cpu.reset(rs.choice(T, R, replace=False), rs.choice(T, T // 2, replace=False) + R)
            k = 40 if R <= 6 else 5
            t0 = time.perf_counter()
            for _ in range(k):
                cpu.step(rs.choice(4, size=(R, 1)))
            row["cpu_ref_1core_random"] = {"step_ms": 1e3 * (time.perf_counter() - t0) / k,
                                           "kind": "reference op sequence (oracle/cpu_ref_coverage.py)"}
            o = oc.CoverageOracle(targets, R, M)
            t0 = time.perf_counter()
            cost, prev = oc.time_matrix(T, o.motion[0] - R, o.motion[1] - R)
            tm = time.perf_counter() - t0
            o.reset(rs.choice(T, R, replace=False), rs.choice(T, T // 2, replace=False) + R)
            t0 = time.perf_counter()
            for _ in range(k):
                cur = o.closest()
                a, _ = oc.greedy_actions(cost, prev, cur, o.visited[R:], oc.action_receivers(cur, o.nbr, o.cnt, R), R)
                o.step(a)
            row["cpu_port_1core_greedy"] = {"step_ms": 1e3 * (time.perf_counter() - t0) / k,
                                            "time_matrix_ms_per_map": 1e3 * tm,
                                            "kind": "port (oracle/coverage.py, NumPy, 1 thread)"}
        out["r%d" % R] = row
    out["note"] = ("per call of env.step(env.controller(...)) on one CoverageEnv, whole episodes after one warm-up "
                   "episode; step_ms leaves the resets out, reset_ms is reset() alone (a new map: its cities from "
                   "np.random, the roads, targets and motion graph on the device; then the start draws) and "
                   "episode_ms_with_reset the whole episode as the reference's driver loop (test.py:43-74) runs it; "
                   "a greedy episode's first step builds the new map's time matrix (first_step_ms); max_nodes 1000 "
                   "(the generated maps hold up to ~650 targets)")
    return out


def bench_greedy(v, targets, R, M, B, K, args):
    """§8f: the greedy expert (controller(greedy=True)) on the same batch: the per-graph
    time-matrix build for all B envs, then expert steps (greedy actions and the step in one
    launch per half batch; fallback robots draw np_random.choice(4) from their env's stream
    on the device, as the reference does, or take action 0 in the "fallback_action0" form)."""
    v.set_targets(targets)  # invalidates every env's time matrix
    v.sync()
    t0 = time.perf_counter()
    v.h.controller_greedy(fetch=False)
    v.sync()
    build = time.perf_counter() - t0
    def loop(step, k):
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        v.sync()
        return time.perf_counter() - t0

    def separate():
        v.h.controller_greedy(fetch=False)
        v.step(resident=True)

    # the fused form: greedy actions from the per-node greedy lists inside the step launch
    # (COV_ACTIONS_GREEDY), the default expert step; then the two-launch form beside it
    state = v.h.robots(0)  # (a sync point: the steps below start from the same batch)
    loop(lambda: v.step(greedy=True), 20)
    el = loop(lambda: v.step(greedy=True), K)
    el_sep = loop(separate, K)
    el0 = loop(lambda: v.step(greedy=True, fallback="zero"), K)
    # in episodes: reset every 75 steps (the reference's EPISODE_LENGTH), resets untimed,
    # so most steps see unvisited targets nearby (the long run above is mostly the
    # all-visited tail, where every robot falls back); each reset seeds every env's
    # np_random (seed + b, after reset's draws) and the fallback draws continue it
    ep_t, ep_k, z_t = 0.0, 0, 0.0
    for e in range(4):
        v.reset(seed=100 + e)
        v.sync()
        ep_t += loop(lambda: v.step(greedy=True), 75)
        ep_k += 75
    for e in range(4):
        v.reset(seed=100 + e)
        v.sync()
        z_t += loop(lambda: v.step(greedy=True, fallback="zero"), 75)
    # the reference's own semantics in episodes: the fallback robots' actions drawn on the
    # host (np_random.choice(4) per robot in robot order, coverage.py:863-864), so every
    # step is the greedy kernel, a device-to-host copy of the actions and flags, the draws,
    # the upload and the step
    rng = np.random.RandomState(17)
    fa_t, fa_k = 0.0, 0
    for e in range(4):
        v.reset(seed=100 + e)
        v.sync()
        t0 = time.perf_counter()
        for _ in range(75):
            a, rnd = v.h.controller_greedy()
            k = np.nonzero(rnd.ravel())[0]
            if len(k):
                a.ravel()[k] = rng.choice(4, size=len(k))
            v.step(a)
        v.sync()
        fa_t += time.perf_counter() - t0
        fa_k += 75
    del state
    # an episode's reset for all envs: its random draws on the device (the default), and
    # the same draws by RandomState loops on the host (bit-identical, tests)
    t0 = time.perf_counter()
    v.reset(seed=500)
    reset_dev = time.perf_counter() - t0
    # whole expert episodes as a data-collection loop runs them: reset (draws on the
    # device) + 75 fused expert steps, for all envs, back to back
    v.sync()
    t0 = time.perf_counter()
    for e in range(4):
        v.reset(seed=600 + e)
        for _ in range(75):
            v.step(greedy=True)
    v.sync()
    episode = (time.perf_counter() - t0) / 4
    # the same episodes with their 75 expert steps in one launch (cov_step_expert: each env's
    # workgroup steps its env 75 times; bit-exact with the launch per step, GPU tests)
    v.sync()
    t0 = time.perf_counter()
    for e in range(4):
        v.reset(seed=600 + e)
        v.expert_steps(75, fetch=False)
    v.sync()
    episode_one = (time.perf_counter() - t0) / 4
    t0 = time.perf_counter()
    v.reset(seed=500, draws="host")
    reset_host = time.perf_counter() - t0
    # the same episodes with a new map for every env at every reset, as each reference
    # reset() draws one (coverage.py:378-397): the maps, their motion graphs and time
    # matrices (built on the episode's first expert step), the reset draws and 75 expert
    # steps, for 512 distinct maps per episode
    v.generate_maps(map_seed=8)
    v.reset(seed=699)
    v.step(greedy=True)
    v.sync()
    t0 = time.perf_counter()
    for e in range(3):
        v.reset(seed=700 + e, new_maps=True)
        for _ in range(75):
            v.step(greedy=True)
    v.sync()
    episode_new = (time.perf_counter() - t0) / 3
    t0 = time.perf_counter()
    v.reset(seed=710, new_maps=True)
    v.h.controller_greedy(fetch=False)  # the time matrices and greedy lists of the new maps
    v.sync()
    reset_tm_new = time.perf_counter() - t0
    out = {"time_matrix_ms_all_envs": 1e3 * build, "envs": B, "n_targets": len(targets),
           "reset_ms_all_envs": 1e3 * reset_dev, "reset_ms_all_envs_host_draws": 1e3 * reset_host,
           "expert_episode_ms_all_envs": 1e3 * episode, "expert_env_episodes_per_s": B / episode,
           "expert_episode_ms_all_envs_one_launch": 1e3 * episode_one,
           "expert_episode_ms_all_envs_new_maps": 1e3 * episode_new,
           "expert_env_episodes_per_s_new_maps": B / episode_new,
           "new_maps_reset_and_time_matrices_ms_all_envs": 1e3 * reset_tm_new,
           "expert_step_ms_in_episodes": 1e3 * ep_t / ep_k,
           "expert_robot_steps_per_s_in_episodes": R * B * ep_k / ep_t,
           "expert_step_ms_in_episodes_fallback_action0": 1e3 * z_t / ep_k,
           "expert_step_ms_in_episodes_host_fallback_draws": 1e3 * fa_t / fa_k,
           "expert_step_ms_steady_all_visited": 1e3 * el / K,
           "expert_step_ms_steady_all_visited_fallback_action0": 1e3 * el0 / K,
           "expert_step_ms_two_launches_steady_fallback_action0": 1e3 * el_sep / K,
           "note": "expert step = controller(greedy=True) + step for every env, the reference's semantics. "
                   "in_episodes (the headline): reset every 75 steps (EPISODE_LENGTH), resets untimed; the greedy "
                   "actions come from per-node greedy lists (or, with at most 32 targets unvisited, the direct "
                   "minimum over them) inside the step's own launch (COV_ACTIONS_GREEDY), and the fallback robots "
                   "draw np_random.choice(4) from their env's MT19937 stream on the device in robot order "
                   "(COV_GREEDY_RNG, bit-exact with the host RandomState); fallback_action0: the same with "
                   "action 0 for the fallback robots; host_fallback_draws: the greedy kernel, the actions and "
                   "flags to the host, np_random draws there, the upload and the step; steady_all_visited: "
                   "thousands of steps from one reset, every target visited (every robot draws)"}
    if not args.no_cpu_baseline:
        from oracle import coverage as oc
        o = oc.CoverageOracle(targets, R, M)
        t0 = time.perf_counter()
        cost, prev = oc.time_matrix(len(targets), o.motion[0] - R, o.motion[1] - R)
        out["cpu_time_matrix_s_per_env"] = time.perf_counter() - t0
        rs = np.random.RandomState(0)
        T = len(targets)
        o.reset(rs.choice(T, R, replace=False), rs.choice(T, T // 2, replace=False) + R)
        t0 = time.perf_counter()
        for _ in range(5):
            cur = o.closest()
            a, _ = oc.greedy_actions(cost, prev, cur, o.visited[R:], oc.action_receivers(cur, o.nbr, o.cnt, R), R)
            o.step(a)
        out["cpu_expert_step_ms_per_env"] = 1e3 * (time.perf_counter() - t0) / 5
        out["cpu_kind"] = "port (oracle/coverage.py, NumPy, 1 thread)"
    return out


# ------------------------------------------------------------------ multi-rank launch
def visible_gpus():
    """GPUs this process could open, counted WITHOUT initialising HIP: KFD topology nodes
    with SIMDs whose DRM render node is accessible, capped by the *_VISIBLE_DEVICES masks.
    None when the topology cannot be read (the workers then fail loudly at device open)."""
    import glob
    topo = os.environ.get("GYMFLOCK_KFD_TOPOLOGY", "/sys/class/kfd/kfd/topology")  # tests point it elsewhere
    props = glob.glob(os.path.join(topo, "nodes", "*", "properties"))
    if not props:
        return None
    n = 0
    for path in props:
        try:
            with open(path) as f:
                kv = dict(ln.split()[:2] for ln in f if len(ln.split()) >= 2)
        except OSError:
            continue
        if int(kv.get("simd_count", "0")) <= 0:
            continue
        minor = kv.get("drm_render_minor")
        if minor is not None and not os.access("/dev/dri/renderD%s" % minor, os.R_OK | os.W_OK):
            continue
        n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([t for t in v.split(",") if t.strip()]))
    return n


def _free_port_pair():
    """A port P with P and P + 1 free on 127.0.0.1 (MASTER_PORT and the host channel)."""
    import socket
    for _ in range(64):
        a = socket.socket()
        a.bind(("127.0.0.1", 0))
        p = a.getsockname()[1]
        b = socket.socket()
        try:
            b.bind(("127.0.0.1", p + 1))
            return p
        except OSError:
            continue
        finally:
            a.close()
            b.close()
    raise RuntimeError("no free port pair")


def launch(args):
    """--gpus N without WORLD_SIZE: spawn N workers (this script, RANK/LOCAL_RANK/
    WORLD_SIZE/MASTER_* set), relay rank 0's JSON line; non-zero exit if N exceeds the
    visible GPUs, if any worker fails or the run outlasts --launch-timeout. The parent
    never touches the GPU (visible_gpus reads sysfs only)."""
    import secrets
    import signal
    import subprocess
    import threading
    n = args.gpus
    if not args.dry_host:
        vis = visible_gpus()
        if vis is not None and n > vis:
            log("bench.py: --gpus %d but only %d GPU(s) are visible" % (n, vis))
            return 2
    port = _free_port_pair()
    token = secrets.token_hex(16)
    children = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GYMFLOCK_HOST_TOKEN=token)
        env.pop("GYMFLOCK_HOST_PORT", None)
        children.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                         stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                         start_new_session=True))
    out = []
    reader = threading.Thread(target=lambda: out.append(children[0].stdout.read()), daemon=True)
    reader.start()
    deadline = time.monotonic() + args.launch_timeout
    failed = None
    while failed is None:
        codes = [c.poll() for c in children]
        bad = ["rank %d exited with %d" % (r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed = "; ".join(bad)
        elif all(c == 0 for c in codes):
            break
        elif time.monotonic() > deadline:
            failed = "timed out after %.0f s" % args.launch_timeout
        else:
            time.sleep(0.05)
    if failed is not None:
        for sig in (signal.SIGTERM, signal.SIGKILL):
            for c in children:
                if c.poll() is None:
                    try:
                        os.killpg(c.pid, sig)  # the worker's own session (start_new_session)
                    except ProcessLookupError:
                        pass
            t_end = time.monotonic() + 10
            while time.monotonic() < t_end and any(c.poll() is None for c in children):
                time.sleep(0.05)
        log("bench.py launcher: %s; the %d-rank run failed" % (failed, n))
        return 1
    reader.join(timeout=30)
    lines = [ln for ln in (out[0] if out else b"").decode(errors="replace").splitlines() if ln.startswith("{")]
    if not lines:
        log("bench.py launcher: rank 0 printed no JSON line")
        return 1
    print(lines[-1], flush=True)
    return 0


def dry_host(args, world, rank):
    """--dry-host: the multi-rank path's host side with no GPU and no HIP library: the
    host-channel rendezvous (token checked), the shard-size exchange, K timed steps of the
    CPU oracle on this rank's envs between barriers, the reward all-gather over the host
    channel in the RCCL path's padded block layout (every rank ships the largest shard's
    width, shard.pad_block; shard.unpad_gathered restores the env order) and every rank's
    whole-vector check. Rank 0 prints a line shaped like the GPU one (n_gpus, per-rank ms,
    gathered_rewards_ok)."""
    from gym_flock.hostgroup import HostGroup
    from gym_flock.init_states import synthetic_state
    from gym_flock.shard import check_gathered, exchange_shard_sizes, pad_block, unpad_gathered
    from oracle import flocking as orc
    group = HostGroup.from_env(timeout=120.0)
    ranks = Ranks(group)
    N, K = args.n_agents, args.steps
    B = args.n_envs + (1 if args.dry_host_uneven and rank == world - 1 else 0)
    sizes = exchange_shard_sizes(group, B)
    W = max(sizes)

    def padded_gather(local):  # the RCCL gathers' block layout, over the host channel
        blk = pad_block(local, W).reshape(W, -1)
        parts = [np.frombuffer(p, np.float64).reshape(W, -1) for p in group.allgather_bytes(blk.tobytes())]
        return unpad_gathered(parts, sizes, axis=0)

    xs = [synthetic_state(N, rank * B + b) for b in range(B)]
    us = [np.random.RandomState(10_000 + rank * B + b).uniform(-1, 1, size=(N, 2)).astype(np.float32)
          for b in range(B)]
    rew = np.zeros(B)

    def step():
        for b in range(B):
            r = orc.step(xs[b], us[b])
            xs[b], rew[b] = r["x"], r["reward"]

    for _ in range(args.warmup):
        step()
    group.barrier()
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    el = time.perf_counter() - t0
    group.barrier()
    every = ranks.gather(el)
    gathered = padded_gather(rew).ravel()
    if args.dry_host_corrupt and rank == 1:
        gathered[0] += 1e-9
    _, ok = check_gathered(group, gathered, rew)
    # the get_stats aggregates: per-env [mean vel_diffs, mean min_dists], host channel
    summ = np.array([[st["vel_diffs"].mean(), st["min_dists"].mean()] for st in map(orc.stats, xs)]).reshape(B, 2)
    gstats = padded_gather(summ)
    _, sok = check_gathered(group, gstats, summ)
    group.close()
    if rank == 0:
        print(json.dumps({"metric": "agent-steps/sec (dry host: CPU oracle, no GPU)", "value": world * B * N * K / max(every),
                          "unit": "agent-steps/s", "n_gpus": world, "steps": K, "warmup": args.warmup,
                          "ms_per_step": 1e3 * max(every) / K,
                          "per_rank_ms_per_step": [1e3 * e / K for e in every],
                          "gathered_rewards_ok": ok, "gathered_stats_ok": sok, "dry_host": True,
                          "shard_sizes": sizes,
                          "config": {"n_agents": N, "envs_per_gpu": B, "global_envs": sum(sizes)}}), flush=True)
    if not (ok and sok):
        raise SystemExit("gathered rewards or stats differ from the ranks' local values")


def cpu_share():
    """The host CPUs the CPU baseline may use: nproc (os.cpu_count), this process's
    affinity set, and the cgroup CPU quota; the usable share is the smallest."""
    nproc = os.cpu_count() or 1
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(nproc))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    use = min([len(aff)] + ([quota] if quota else []))
    return {"nproc": nproc, "affinity": len(aff), "cgroup_quota": quota, "use": use, "cores": aff[:use]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["flocking", "coverage"], default="flocking")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n-agents", type=int, default=1024)
    ap.add_argument("--n-envs", type=int, default=256, help="envs per GPU")
    ap.add_argument("--metrics-every", type=int, default=8,
                    help="steps per reward all-gather (N>1, at most 64); each collective carries all those steps")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--clock-warmup-ms", type=float, default=300.0,
                    help="untimed wall time of steps before the warmup steps (reported)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="processes of the all-cores CPU baseline (default: the usable CPU share, "
                         "min(nproc, affinity, cgroup quota), capped by OMP_NUM_THREADS when set)")
    ap.add_argument("--cpu-worker", type=float, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--pin-core", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="seconds the --gpus N launcher waits for its workers")
    ap.add_argument("--dry-host", action="store_true",
                    help="multi-rank host path only (spawn, rendezvous, reward check) with the CPU oracle; no GPU")
    ap.add_argument("--dry-host-uneven", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-host-corrupt", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--seed", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--no-controller-line", action="store_true")
    ap.add_argument("--no-packed-line", action="store_true")
    ap.add_argument("--no-host-actions-line", action="store_true")
    ap.add_argument("--no-knn-line", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the configs[3] (Coverage) and configs[4] (N=8192) sub-objects")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the multi-rank path (host channel + RCCL reward all-gather) even at 1 rank")
    args = ap.parse_args()
    if not 1 <= args.metrics_every <= 64:
        ap.error("--metrics-every must be in [1, 64] (the reward ring holds 64 steps)")
    if args.cpu_worker is not None:
        return cpu_worker(args.n_agents, args.cpu_worker, args.seed, args.pin_core)
    if args.workload == "coverage":
        print(json.dumps(dict(bench_config4(args, with_greedy=True), n_gpus=1)), flush=True)
        return

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log("bench.py: WORLD_SIZE=%d but --gpus %d: one rank per GPU is required" % (world, args.gpus))
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_host:
        return dry_host(args, world, rank)
    multi = world > 1 or args.force_dist
    group = None
    if multi:
        from gym_flock.hostgroup import HostGroup
        group = HostGroup.from_env()
    ranks = Ranks(group)

    from gym_flock.shard import check_gathered, init_rccl_gather, rccl_report
    from gym_flock.vec import VecFlockingRelative

    N, B, K, W = args.n_agents, args.n_envs, args.steps, args.warmup
    t_setup = time.perf_counter()
    env = VecFlockingRelative(B, N, device=local_rank, env_offset=rank * B)
    x_init = env.reset(seed=0)
    u = np.random.RandomState(1234 + rank).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    env.set_actions(u)
    warm = clock_warmup(lambda: env.step(resident=True), env.sync, args.clock_warmup_ms)
    env.set_state(x_init)
    gather = None
    if multi:
        # after the clock warmup: the first reward gather ships the steps since init
        # RCCL prints a version banner on the process's stdout at communicator init; the
        # bench's stdout carries only the JSON line, so fd 1 points at stderr meanwhile
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            gather = init_rccl_gather(group, env.h, world, rank)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    log("setup %.1fs: N=%d B=%d per GPU, world=%d" % (time.perf_counter() - t_setup, N, B, world))
    ungathered = [0]  # steps since the last reward all-gather

    def plain(s):
        env.step(resident=True)
        ungathered[0] += 1
        if gather is not None and (s + 1) % args.metrics_every == 0:
            gather.issue()  # every step since the previous issue, in one collective
            ungathered[0] = 0
    if gather is not None:
        # RCCL's initialisation leaves the GPU idle long enough for its clocks to drop back
        # (the timed window then ran ~20 % slower at one rank, profiles/r05/forcedist_rewarm.txt):
        # step again, gathering as the timed loop does, a fixed count on every rank (the
        # collectives must match), then restore the synthetic init
        for s in range(REWARM_STEPS):
            plain(s)
        if ungathered[0]:  # the next gather must not span more than the ring's 64 steps
            gather.issue()
            ungathered[0] = 0
        env.sync()
        env.set_state(x_init)
        warm["steps_after_comm_init"] = REWARM_STEPS
    for s in range(W):
        plain(s)
    per_rank = []
    elapsed, kernel_ms = timed(env, ranks, K, plain, per_rank)

    extra = {}
    if gather is not None:
        # RCCL's own view of the ranks, checked on rank 0's line: one communicator of
        # world ranks, user ranks 0..world-1, a distinct GPU (PCI bus id) per rank
        extra["rccl"] = rccl_report(group, gather, world)
        if ungathered[0]:
            gather.issue()  # the steps after the last in-loop all-gather
        allr = gather.result()  # (steps, total envs), the last row is the latest step
        _, every = check_gathered(group, allr[-1], env.rewards())
        extra["gathered_rewards_ok"] = every
        extra["gathered_rewards_check"] = ("every rank compared the whole gathered (world x B) vector of the last "
                                           "step with the ranks' local rewards sent over the host channel")
        # the optional get_stats aggregates: per-env means, all-gathered once
        gather.issue_stats()
        _, sok = check_gathered(group, gather.stats_result(), env.stats_summary())
        extra["gathered_stats_ok"] = sok

    # closed-loop step + fused controller (u = previous controller output), same workload
    if not args.no_controller_line:
        env.reset(x=x_init)
        env.controller()
        clock_warmup(lambda: env.step(expert=True, controller=True), env.sync, 50.0)
        env.reset(x=x_init)
        env.controller()
        for _ in range(min(W, 5)):
            env.step(expert=True, controller=True)
        ec, cms = timed(env, ranks, K, lambda s: env.step(expert=True, controller=True))
        cb = B * (step_bytes(N) + N * 8 * 2)  # + the controller's output (read back as the next u)
        cach = cb / (cms * 1e-3) / 1e9 if cms > 0 else 0.0
        extra["step_with_controller"] = {"value": world * B * N * K / ec, "unit": "agent-steps/s",
                                         "ms_per_step": 1e3 * ec / K, "region_ms_per_step": cms,
                                         "algorithmic_bytes_per_step": cb,
                                         "roofline": {"bound": "hbm", "achieved": cach, "peak": HBM_PEAK_GBS,
                                                      "unit": "GB/s", "frac": cach / HBM_PEAK_GBS,
                                                      "traffic": load_traffic("ctrl_1024x256"),
                                                      "kernel": "flock_step_kernel<DYN,f64 u,CTRL>"}}

    # packed output mode: adjacency bits + degree instead of the dense rows
    if not args.no_packed_line:
        clock_warmup(lambda: env.step(resident=True, network="packed"), env.sync, 50.0)
        env.reset(x=x_init)
        env.step(resident=True, network="packed")
        ep, pk_ms = timed(env, ranks, K, lambda s: env.step(resident=True, network="packed"))
        wn = (N + 63) // 64
        pk_bytes = B * (8 * N * wn + 4 * N + 96 * N + 8)
        pach = pk_bytes / (pk_ms * 1e-3) / 1e9 if pk_ms > 0 else 0.0
        extra["packed_network"] = {
            "value": world * B * N * K / ep, "unit": "agent-steps/s", "ms_per_step": 1e3 * ep / K,
            "region_ms_per_step": pk_ms, "algorithmic_bytes_per_step": pk_bytes,
            "roofline": {"bound": "hbm", "achieved": pach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": pach / HBM_PEAK_GBS, "traffic": load_traffic("packed_1024x256"),
                         "kernel": "flock_step_kernel<DYN,f32 u> (packed output)"},
            "note": "adjacency as bits (N*ceil(N/64)*8 B) + int32 degree per env instead of the dense "
                    "float32 network; the pair work, not HBM, bounds this mode"}

    # the same step with host actions: the (B,N,2) float32 actions copied from pageable host
    # memory every step (the PCIe-inclusive rate of a trainer that hands actions over per
    # step; the headline keeps them resident in HBM)
    if not args.no_host_actions_line:
        clock_warmup(lambda: env.step(u), env.sync, 50.0)  # as the other lines
        env.reset(x=x_init)
        for _ in range(max(1, min(W, 5))):  # untimed, as the other lines' warmup steps
            env.step(u)
        calls = []

        def host_step(s):
            c0 = time.perf_counter()
            env.step(u)
            calls.append(1e6 * (time.perf_counter() - c0))

        eh, _ = timed(env, ranks, K, host_step)
        extra["host_actions"] = {
            "value": world * B * N * K / eh, "unit": "agent-steps/s", "ms_per_step": 1e3 * eh / K,
            "ratio_to_plain_step": eh / elapsed, "action_bytes_per_step": int(u.nbytes),
            "call_us_first": [round(c, 1) for c in calls[:6]], "call_us_median": float(np.median(calls)),
            "note": "PCIe-inclusive: env.step(u) with a host (B,N,2) float32 action array each step, uploaded "
                    "on the handle's action stream into one of two device buffers while the previous step "
                    "runs (fe_step returns once its copy is done, not its step); outputs stay in HBM"}

    # Flocking-v0 (§8f rank 1): the same step plus the 7-nearest-neighbour observation
    # (flocking.py:20-25), dense network kept; a second handle with n_neighbors=7. The
    # first handle is closed first so the lines stay independent (a kNN handle runs two
    # HIP streams, so two handles fit the process's 4 hardware queues: 235.2 vs 235.7 us
    # with a second live handle, profiles/r03/knn_second_handle.txt)
    env.close()
    if not args.no_knn_line:
        envk = VecFlockingRelative(B, N, device=local_rank, env_offset=rank * B, n_neighbors=7)
        envk.set_state(x_init)
        envk.set_actions(u)
        clock_warmup(lambda: envk.step(resident=True, knn=True), envk.sync, 50.0)
        envk.reset(x=x_init)
        for _ in range(min(W, 5)):
            envk.step(resident=True, knn=True)
        ek, kk_ms = timed(envk, ranks, K, lambda s: envk.step(resident=True, knn=True))
        # the step's bytes + per agent idx (7 x int32), obs (28 x float32) and the k-th
        # nearest r2 (float32) written, the history r2 read
        kb = B * (step_bytes(N) + N * (7 * 4 + 28 * 4 + 4 + 4))
        kach = kb / (kk_ms * 1e-3) / 1e9 if kk_ms > 0 else 0.0
        extra["flocking_v0_knn7"] = {
            "value": world * B * N * K / ek, "unit": "agent-steps/s", "ms_per_step": 1e3 * ek / K,
            "region_ms_per_step": kk_ms, "ratio_to_plain_step": ek / elapsed,
            "algorithmic_bytes_per_step": kb,
            "roofline": {"bound": "hbm", "achieved": kach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": kach / HBM_PEAK_GBS, "traffic": load_traffic("knn7_1024x256"),
                         "kernel": "flock_step_kernel<DYN,f32 u,KN=7> (+ rim flock_knn_kernel on the step streams)"},
            "note": "Flocking-v0 step: FlockingRelative step + 7-NN observation (idx + obs), from the "
                    "synthetic init under the same random actions"}
        envk.close()

    if rank == 0:
        value = world * B * N * K / elapsed
        line = {
            "metric": "agent-steps/sec (N_agents×N_envs×steps/s), FlockingRelative N=%d" % N,
            "value": value,
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "clock_warmup": warm,
            "ms_per_step": 1e3 * elapsed / K,
            "per_rank_ms_per_step": [1e3 * e / K for e in per_rank],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (random-init swarms, SURVEY.md §8d; float32 actions U(-1,1) resident in HBM)",
            "config": {"workload": "FlockingRelative-v0 step(), N=%d agents x %d envs per GPU%s"
                                   % (N, B, CONFIG_TAG.get((N, B, world), "")),
                       "n_agents": N, "envs_per_gpu": B, "global_envs": world * B,
                       "outputs": "network (N,N) f32 + state_values (N,6) f32 + reward, in HBM",
                       "parallelism": (("env-sharded dp%d, RCCL reward all-gather of every step, one collective "
                                        "per %d steps" % (world, args.metrics_every)) if gather is not None else
                                       "env-sharded dp%d, no collective ran (one rank: the reward all-gather "
                                       "runs at N>1 or with --force-dist)" % world)},
            "roofline": flock_roofline(N, B, kernel_ms, 2 if B >= 2 else 1),
        }
        line.update(extra)
        from gym_flock import _native as nat
        line["runtime"] = nat.runtime_info()  # the HIP runtime and RCCL this process measured on
        if world == 1 and not args.no_other_configs:
            log("config 4 (Coverage R=200 x 512, with the greedy expert and per-episode maps)...")
            line["coverage_config4"] = bench_config4(args, with_greedy=True)
            log("config 5 (N=8192 x 32)...")
            line["n8192_config5"] = bench_config5(args)
            log("drop-in single-env path (N=100, 1024)...")
            line["dropin"] = bench_dropin(args)
            log("drop-in Coverage env (R=6, 200)...")
            line["dropin_coverage"] = bench_dropin_coverage(args)
        if not args.no_cpu_baseline:
            # rank 0 after the timed region (the other ranks are done stepping): the same
            # host-core baseline beside every world size's line
            log("cpu baseline (cpu_ref, 1 core, ~%.0fs)..." % args.cpu_seconds)
            line["cpu_baseline"] = flock_cpu_baseline(N, args.cpu_seconds, args.cpu_procs or None)
        print(json.dumps(line), flush=True)
    if group is not None:
        group.close()


if __name__ == "__main__":
    main()
