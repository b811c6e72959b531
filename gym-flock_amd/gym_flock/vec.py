"""Batched FlockingRelative / Flocking-v0: B independent envs stepped by one launch.

This is the data-parallel form of the reference's per-env loop (one
FlockingRelativeEnv.step per env per step, flocking_relative.py:91-109). Outputs
stay in device memory; the getters copy to the host on demand, so a trainer that
only needs rewards or a few envs' observations never pays for the (B,N,N) network
transfer.
"""
import numpy as np

from . import _native as nat
from .init_states import synthetic_batch


# fe_variant presets of the registered flocking variants (include/gymflock.h)
VARIANTS = {
    "relative": {},
    "leader": dict(u_scale=1.0, n_frozen=2),                      # flocking_leader.py
    "obstacle": dict(u_scale=1.0, n_frozen=4, n_vel_zero=4),      # flocking_obstacle.py
    "stochastic": dict(u_scale=6.0, u_clip=0.5, x_scale=6.0, ctrl_clip=0.5),  # flocking_stoch.py
    "twoflocks": {},                                              # reset only
}


class VecFlockingRelative:
    """B FlockingRelative-v0 envs of N agents on one GPU.

    env_offset: global index of this shard's first env (seeds are env_offset + b),
    so a batch sharded over ranks reproduces the single-device batch.
    variant: a VARIANTS key or a dict of fe_variant fields (flocking variants).
    """

    def __init__(self, n_envs, n_agents, comm_radius=0.9, dt=0.01, v_max=5.0,
                 action_scalar=10.0, mean_pooling=True, centralized=True, n_neighbors=0,
                 device=0, env_offset=0, variant=None):
        self.n_envs, self.n_agents = int(n_envs), int(n_agents)
        self.v_max = v_max
        self.env_offset = int(env_offset)
        self.h = nat.FlockHandle(n_agents, n_envs, comm_radius, dt, action_scalar,
                                 mean_pooling, centralized, n_neighbors, device)
        v = VARIANTS[variant] if isinstance(variant, str) else variant
        if v:
            self.h.set_variant(**v)

    # ------------------------------------------------------------------- state
    def reset(self, seed=0, x=None):
        """Synthetic init for envs seed+env_offset+b, or a given (B,N,4)."""
        if x is None:
            x = synthetic_batch(self.n_envs, self.n_agents, seed + self.env_offset, self.v_max)
        self.h.set_state(x)
        self.h.compute_helpers()
        return x

    def set_state(self, x):
        self.h.set_state(x)

    def get_state(self):
        return self.h.get_state()

    # ---------------------------------------------------------------- hot path
    def step(self, u=None, controller=False, knn=False, network=True, expert=False,
             resident=False, device_ptr=None, dt=None):
        """Advance every env one step.

        network: True (dense (N,N) rows), False (none), "packed" (adjacency bits +
        degree only) or "both".
        u: (B,N,2) host actions (float32 or float64 arithmetic like the reference); or
        expert=True to feed back the previous controller() output (closed loop); or
        resident=True to reuse the actions last given to set_actions(); or
        device_ptr=<int> for a device buffer of float32 actions.
        dt: per-env (B,) time step for this and later steps (the stochastic variant).
        Asynchronous: returns once the launch is queued (host actions are copied first).
        """
        if dt is not None:
            self.h.set_dt(dt)
        flags = 0
        if controller:
            flags |= nat.FE_WITH_CONTROLLER
        if knn:
            flags |= nat.FE_WITH_KNN
        if network == "packed":  # adjacency bits + degree instead of the dense (N,N) rows
            flags |= nat.FE_PACKED_NETWORK | nat.FE_NO_NETWORK
        elif network == "both":
            flags |= nat.FE_PACKED_NETWORK
        elif not network:
            flags |= nat.FE_NO_NETWORK
        if expert:
            self.h.step(None, flags | nat.FE_U_EXPERT)
        elif resident:
            self.h.step(None, flags | nat.FE_U_RESIDENT)
        elif device_ptr is not None:
            self.h.step(device_ptr, flags | nat.FE_U_DEVICE)
        else:
            self.h.step(u, flags)

    def set_actions(self, u):
        self.h.set_actions(u)

    def controller(self, centralized=None):
        return self.h.controller(centralized)

    # ----------------------------------------------------------------- outputs
    def state_values(self, env=None):
        return self.h.state_values(env)

    def network(self, env=None):
        return self.h.network(env)

    def rewards(self):
        return self.h.rewards()

    def network_packed(self, env=None):
        """Adjacency bits and degrees of the last step(network="packed" or "both")."""
        return self.h.network_packed(env)

    def controls(self, env=None):
        return self.h.controls(env)

    def knn(self, env=None):
        return self.h.knn(env)

    def stats(self, env=0):
        return self.h.stats(env)

    def stats_summary(self):
        """(B, 2) per-env np.mean(vel_diffs), np.mean(min_dists) (get_stats, :136-143)."""
        return self.h.stats_summary()

    def sync(self):
        self.h.sync()

    def close(self):
        self.h.close()


class VecCoverage:
    """B Coverage-v0 envs (R robots each) on one GPU, one workgroup per env.

    Each env gets its own target graph (set_targets(env=b)) or all share one
    (env=-1); reset() draws starts and the unvisited set per env from
    np.random.RandomState(seed + env_offset + b) in the reference's order.
    """

    def __init__(self, n_envs, n_robots, max_nodes=1000, episode_length=75, res=5.5,
                 frac_active_targets=0.5, device=0, env_offset=0):
        self.n_envs, self.n_robots = int(n_envs), int(n_robots)
        self.frac = frac_active_targets
        self.env_offset = int(env_offset)
        self.h = nat.CoverageHandle(n_robots, n_envs, max_nodes, episode_length, res, None, device)
        self.n_targets = np.zeros(self.n_envs, np.int64)
        self._rngs = None          # host-held np_random streams (else on the device)
        self._dev_streams = False  # the device holds every env's np_random stream

    def set_targets(self, targets, env=-1):
        self.h.set_targets(targets, env)
        if env < 0:
            self.n_targets[:] = len(targets)
        else:
            self.n_targets[env] = len(targets)

    def generate_maps(self, map_seed=None):
        """A new target map for every env on the device (coverage.py:516-527, as each
        reference reset() draws one): env b's cities come from its own map stream, seeded
        np.random.seed(map_seed + env_offset + b) when map_seed is given, else continued
        from its previous map, as the reference's global np.random continues from one
        reset to the next. Returns (n_targets (B,), status (B,))."""
        seed = None if map_seed is None else int(map_seed) + self.env_offset
        n, st, _ = self.h.generate_maps(map_seed=seed)
        self.n_targets[:] = n
        return n, st

    def targets(self, env):
        """Env `env`'s current map, (n_targets, 2) float64 (cov_get_targets)."""
        return self.h.targets(env, int(self.n_targets[env]))

    def reset(self, seed=0, draws="device", new_maps=False, map_seed=None):
        """Env b is a reference env whose np_random was seeded seed + env_offset + b: its
        reset draws (coverage.py:405-424), then its stream continues on the device for the
        greedy expert's fallback draws (step(greedy=True)); np_random(b) reads it back.
        draws="device" (cov_reset_seeded): the draws run on the device, one wave per env;
        "host": RandomState loops here (~0.5 ms per env), then cov_reset and cov_set_rng.
        Both return (start (B,R) target-local, visited (B, max_nodes-R)), bit-identical.
        new_maps: each env first draws a new map on the device (generate_maps(map_seed)),
        as every reference reset() does (:378-397)."""
        if new_maps:
            self.generate_maps(map_seed)
        self._rngs = None
        if draws == "device":
            out = self.h.reset_seeded(seed + self.env_offset, self.frac)
            self._dev_streams = True
            return out
        R, tmax = self.n_robots, self.h.t_max
        start = np.empty((self.n_envs, R), np.int32)
        visited = np.ones((self.n_envs, tmax), np.uint8)
        rngs = []
        for b in range(self.n_envs):
            rs = np.random.RandomState(seed + self.env_offset + b)
            T = int(self.n_targets[b])
            start[b] = rs.choice(np.arange(T), size=(R,), replace=False)
            drop = rs.choice(np.arange(T) + R, size=(int(T * self.frac),), replace=False)
            visited[b, drop - R] = 0
            rngs.append(rs)
        self.h.reset(start, visited)
        if R <= 624:  # device draws (COV_GREEDY_RNG): one key regeneration per step at most
            self.h.set_rng(rngs)
            self._dev_streams = True
        else:
            self._rngs, self._dev_streams = rngs, False
        return start, visited

    def _device_draws(self):
        """Whether the fused greedy step can draw the fallback robots' np_random.choice(4)
        on the device (COV_GREEDY_RNG): the streams live there, n_robots <= 624 (one key
        regeneration per step) and the per-node greedy lists exist (max_nodes - n_robots
        <= 1024)."""
        return self._dev_streams and self._rngs is None and self.n_robots <= 624 and self.h.t_max <= 1024

    def _host_rngs(self):
        """The envs' np_random streams as host RandomStates (read back from the device the
        first time; the host keeps them from then on, until the next reset)."""
        if self._rngs is None:
            if not self._dev_streams:
                raise nat.GymFlockError(nat.GF_ESTATE, "reset first (no np_random streams)")
            keys, pos = self.h.get_rng()
            self._rngs = []
            for b in range(self.n_envs):
                rs = np.random.RandomState()
                rs.set_state(("MT19937", keys[b], int(pos[b])))
                self._rngs.append(rs)
            self._dev_streams = False
        return self._rngs

    def np_random(self, env):
        """Env `env`'s np_random after the fallback draws of the steps so far (a RandomState
        continuing the device stream, or the host one)."""
        if self._rngs is not None:
            return self._rngs[env]
        keys, pos = self.h.get_rng()
        rs = np.random.RandomState()
        rs.set_state(("MT19937", keys[env], int(pos[env])))
        return rs

    def step(self, actions=None, resident=False, greedy=False, fallback="draw"):
        """actions (B,R); or resident=True (the last set/greedy actions); or greedy=True
        (controller(greedy=True), coverage.py:800-872, computed in the step's own launch).
        fallback: robots the reference hands to np_random.choice(4) (:861-864) draw it from
        their env's stream ("draw", the reference's semantics: on the device inside the
        step when _device_draws(), else the greedy kernel, the draws on the host in robot
        order and a resident step) or take action 0 ("zero"); include/gymflock.h
        COV_ACTIONS_GREEDY, COV_GREEDY_RNG."""
        if resident or greedy:
            if greedy and fallback == "draw" and not self._device_draws():
                a, rnd = self.h.controller_greedy()
                if rnd.any():
                    rngs = self._host_rngs()
                    for b in np.nonzero(rnd.any(axis=1))[0]:
                        k = np.nonzero(rnd[b])[0]
                        a[b, k] = rngs[b].choice(4, size=len(k))
                    self.h.set_actions(a)
                rc = self.h._step_resident()
            elif greedy:
                rc = self.h._step_greedy_rng() if fallback == "draw" else self.h._step_greedy()
            else:
                rc = self.h._step_resident()
            if rc:
                nat.check(rc)
            return
        self.h.step(actions)

    def expert_steps(self, n_steps, fetch=True):
        """n_steps of the reference's greedy expert (controller(greedy=True) with its
        np_random.choice(4) fallback draws, then step) for every env in ONE launch
        (cov_step_expert): the same states, rewards and streams as n_steps calls of
        step(greedy=True), for expert rollouts. Needs the streams on the device (a reset with
        draws="device", or R <= 624 with host draws) and the greedy lists
        (max_nodes - n_robots <= 1024). Returns (rewards (n_steps,B), done (n_steps,B)) or
        None with fetch=False."""
        if not self._device_draws():
            raise RuntimeError("expert_steps needs the envs' np_random streams on the device, n_robots <= 624 "
                               "and max_nodes - n_robots <= 1024")
        return self.h.step_expert(n_steps, fetch=fetch)

    def set_actions(self, actions):
        self.h.set_actions(actions)

    def rewards(self):
        return self.h.rewards()

    def obs(self, env=0):
        return self.h.obs(env)

    def flat_obs(self, f32=False, device_ptr=None):
        """Every env's observation as one FlattenDictWrapper row (B, 15*max_nodes + 1)."""
        return self.h.flat_obs(f32, device_ptr)

    def graphs_tuple(self, mask_all=False):
        """The batch as unpack_obs's graph tuple (coverage.py:689-741)."""
        return self.h.graphs_tuple(mask_all)

    def sync(self):
        self.h.sync()

    def close(self):
        self.h.close()
