"""FlockingRelative-v0 on the MI355X engine — drop-in for
gym_flock/envs/flocking/flocking_relative.py of the reference.

Same class name, attributes and method signatures as the reference
(`__init__` :20-66, `params_from_cfg` :68-85, `seed` :87-89, `step` :91-109,
`compute_helpers` :111-134, `get_stats` :136-143, `instant_cost` :145-147,
`reset` :156-192, `controller` :194-212, `render` :234-257, `close` :303). Every
per-step array computation runs in the HIP kernels of libgymflock.so through the
C-ABI (gym_flock._native); nothing here computes pairwise quantities on the host.

Differences a caller can observe:
  - observations are float32 (the reference's observation_space dtype, :59-60); the
    reference returns float64 arrays.
  - `x` is a property backed by device memory: assigning `env.x = arr` uploads,
    reading returns a float64 copy (in-place edits of that copy do not propagate).
  - `diff` / `r2` (N,N,4)/(N,N) are not materialised; `adj_mat` is derived from
    the network.
  - reset() runs the reference's rejection sampler (same global-RNG call order, so
    seeded runs reproduce the reference bit for bit) up to `reset_max_attempts`
    draws, then falls back to a single draw (the reference would loop forever,
    SURVEY.md finding 5); `reset_mode='synthetic'` skips the rejection.
"""
import warnings

import numpy as np

from ... import _native as nat
from ..._spaces import Box, Env, np_random
from ...init_states import draw_swarm


class FlockingRelativeEnv(Env):

    def __init__(self, device=0):
        self.mean_pooling = True  # :27
        self.centralized = True   # :28
        self.nx_system = 4
        self.n_features = 6
        self.nu = 2

        self.n_agents = 100       # :38
        self.comm_radius = 0.9
        self.dt = 0.01
        self.v_max = 5.0
        self.r_max = 1.0

        self.comm_radius2 = self.comm_radius * self.comm_radius
        self.vr = 1 / self.comm_radius2 + np.log(self.comm_radius2)
        self.v_bias = self.v_max

        self.u = None
        self.mean_vel = None
        self.init_vel = None
        self.max_accel = 1
        self.action_scalar = 10.0
        self.device = device
        self.n_neighbors = 0
        self.reset_mode = "reference"
        self.reset_max_attempts = 1000
        # how step() brings (state_values, network, reward) to the host: "direct" = one
        # fe_step_host call: the kernel reads the actions from a page-locked buffer and
        # writes the outputs straight into page-locked arrays from the process's HostPool
        # (fresh arrays to the caller, recycled once released), one launch and one wait;
        # "pooled" = fe_step, then one fe_get_outputs call into pool arrays; "batched" =
        # the same into ordinary numpy arrays; "getters" = three synchronous getters
        self.fetch_mode = "direct"
        # controller() once asked for, every later step also computes the expert action of
        # its resulting state in the same launch, and controller() returns it
        self._want_ctrl = False
        self._ctrl_cache = None
        self._ctrl_key = None  # the handle parameters the cached expert action was computed with
        self._ubuf = None
        self._layout = None  # ((n, ctrl), offsets of the step's page-locked output block)

        self._make_spaces()
        self.fig = None
        self.line1 = None
        self._h = None
        self._hkey = None
        self.state_values = None
        self.state_network = None
        self._reward = None
        self.seed()

    # ------------------------------------------------------------------ config
    def _make_spaces(self):
        self.action_space = Box(low=-self.max_accel, high=self.max_accel,
                                shape=(2 * self.n_agents,), dtype=np.float32)
        self.observation_space = Box(low=-np.inf, high=np.inf,
                                     shape=(self.n_agents, self.n_features), dtype=np.float32)

    def params_from_cfg(self, args):
        """:68-85 (including the r_max *= sqrt(n_agents) compounding on repeat calls)."""
        self.comm_radius = args.getfloat('comm_radius')
        self.comm_radius2 = self.comm_radius * self.comm_radius
        self.vr = 1 / self.comm_radius2 + np.log(self.comm_radius2)
        self.n_agents = args.getint('n_agents')
        self.r_max = self.r_max * np.sqrt(self.n_agents)
        self._make_spaces()
        self.v_max = args.getfloat('v_max')
        self.v_bias = self.v_max
        self.dt = args.getfloat('dt')

    def seed(self, seed=None):
        self.np_random, seed = np_random(seed)
        return [seed]

    def _key(self, centralized=None):
        """The device handle's parameters: the first three fix its buffers, the rest are
        runtime parameters of its launches (fe_set_params); the variant's fields (last)
        are runtime parameters too (fe_set_variant)."""
        c = self.centralized if centralized is None else centralized
        v = self._variant()
        return (self.n_agents, self.n_neighbors, self.device, float(self.comm_radius), float(self._key_dt()),
                float(self.action_scalar), bool(self.mean_pooling), bool(c),
                None if not v else tuple(sorted(v.items())))

    def _key_dt(self):
        """The dt of the handle's launches (a variant that sets dt per step overrides it)."""
        return self.dt

    def _handle(self):
        """The device handle for the current parameters. The reference reads comm_radius,
        dt, action_scalar, mean_pooling and centralized at call time (e.g. :200-201), so a
        change of those between calls keeps the state: the handle takes them as runtime
        parameters. A new n_agents (or device) needs new buffers: the handle is re-created
        and the state starts unset, as the reference's x no longer fits (reset() next)."""
        key = self._key()
        if self._h is not None and key != self._hkey:
            if key[:3] == self._hkey[:3]:
                if key[3:8] != self._hkey[3:8]:
                    self._h.set_params(*key[3:8])
                if key[8] != self._hkey[8]:
                    if key[8]:
                        self._h.set_variant(**dict(key[8]))
                    else:
                        self._h.clear_variant()
                self._hkey = key
            else:
                self._h.close()
                self._h = None
                self._invalidate()
                self._ubuf = None
        if self._h is None:
            self._h = nat.FlockHandle(self.n_agents, 1, self.comm_radius, self._key_dt(),
                                      self.action_scalar, self.mean_pooling, self.centralized,
                                      self.n_neighbors, self.device)
            self._hkey = key
            if key[8]:
                self._h.set_variant(**dict(key[8]))
        return self._h

    def _variant(self):
        """fe_variant fields for subclasses that change the step (flocking variants)."""
        return None

    # ------------------------------------------------------------------- state
    @property
    def x(self):
        if self._h is None:
            return None
        return self._h.get_state(0)

    @x.setter
    def x(self, value):
        value = np.asarray(value, dtype=np.float64)
        assert value.shape == (self.n_agents, self.nx_system), value.shape
        self._handle().set_state(value, env=0)
        self._invalidate()

    def _invalidate(self):
        """The state changed outside step(): the cached expert action is stale."""
        self._ctrl_cache = None

    # ---------------------------------------------------------------- hot path
    def _device_step(self, u):
        """step(u) (u None: compute_helpers) on the device, observations to the host."""
        if self.fetch_mode != "direct":
            h = self._handle()
            if u is None:
                h.compute_helpers()
            else:
                h.step(u[None])
            self._ctrl_cache = None
            self._fetch_obs()
            return
        h = self._handle()
        n = self.n_agents
        f64 = False
        uaddr = None
        if u is not None:
            f64 = nat.u_is_f64(u)
            dt = np.float64 if f64 else np.float32
            if self._ubuf is None or self._ubuf.a.dtype != dt:
                self._ubuf = nat.PinnedArray((n, 2), dt)  # read by the kernel in place
            self._ubuf.a[...] = u
            uaddr = self._ubuf.addr
        # one page-locked block per step: network, controls, reward, state_values (64-byte
        # aligned parts, so the network rows get 16-byte stores); the caller's arrays are
        # made over it, and it returns to the pool once all of them are released
        ctrl = self._want_ctrl
        lay = self._layout
        if lay is None or lay[0] != (n, ctrl):
            o_ct = (4 * n * n + 63) & ~63
            o_rw = o_ct + ((16 * n + 63) & ~63 if ctrl else 0)
            o_sv = o_rw + 64
            lay = self._layout = ((n, ctrl), o_ct, o_rw, o_sv, o_sv + 24 * n)
        _, o_ct, o_rw, o_sv, size = lay
        buf, base = nat.host_pool().block_addr(size)
        if buf is None:  # not page-locked (pool cap): the library copies after the launch
            buf = np.empty(size, np.uint8)
        net = np.ndarray((n, n), np.float32, buf)
        rw = np.ndarray((1,), np.float64, buf, o_rw)
        sv = np.ndarray((n, 6), np.float32, buf, o_sv)
        ct = np.ndarray((n, 2), np.float64, buf, o_ct) if ctrl else None
        if base is None:
            base = buf.ctypes.data
        h.step_host(uaddr, f64, base + o_sv, base, base + o_rw, base + o_ct if ctrl else None)
        self.state_values, self.state_network = sv, net
        self._reward = float(rw[0])
        self._ctrl_cache = ct
        self._ctrl_key = self._hkey

    def _fetch_obs(self):
        h = self._h
        if self.fetch_mode == "getters":
            self.state_values = h.state_values(0)
            self.state_network = h.network(0)
            self._reward = float(h.rewards()[0])
            return
        pool = nat.host_pool() if self.fetch_mode in ("pooled", "direct") else None
        self.state_values, self.state_network, rw = h.outputs(0, pool=pool)
        self._reward = float(rw[0])

    def step(self, u):
        """:91-109 — dynamics, compute_helpers and instant_cost in one device launch (with
        controller() of the new state fused in, once the caller uses the expert)."""
        u = np.asarray(u)
        assert u.shape == (self.n_agents, self.nu)
        self.u = u * self.action_scalar
        self._device_step(u)
        return (self.state_values, self.state_network), self._reward, False, {}

    def compute_helpers(self):
        """:111-134 on the current state."""
        self._device_step(None)

    def instant_cost(self):
        """:145-147 — reward of the current state (computed with the observations)."""
        return self._reward

    @property
    def adj_mat(self):
        return None if self.state_network is None else (self.state_network > 0).astype(float)

    @property
    def adj_mat_mean(self):
        return self.state_network if self.mean_pooling else None

    def get_stats(self):
        """:136-143."""
        vd, md, _ = self._handle().stats(0)
        return {'vel_diffs': vd, 'min_dists': md}

    def controller(self, centralized=None):
        """:194-212 — Turner-2003 expert action (N,2) float64 for the current state. After
        a step (or reset) the action was computed in that launch already: it is returned
        as is (a fresh array; a second call for the same state gets a copy). Otherwise, or
        for other parameters than that launch had (centralized, comm_radius, ...), one
        launch."""
        if centralized is None:
            centralized = self.centralized
        self._want_ctrl = True
        c = self._ctrl_cache
        # the cached action counts only if it was computed with the parameters asked for
        # now (centralized, comm_radius, ... as the env holds them at this call, :200-201)
        if c is not None and self._ctrl_key == self._key(bool(centralized)):
            self._ctrl_cache = c.copy()  # later calls for this state get their own array
            return c
        return self._handle().controller(centralized)[0]

    def potential_grad(self, pos_diff, r2):
        """:214-226 on caller-supplied arrays (the step's own gradient runs fused in the
        device controller): -2 d / r2^2 + 2 d / r2, zero where r2 > comm_radius."""
        grad = -2.0 * np.divide(pos_diff, np.multiply(r2, r2)) + 2 * np.divide(pos_diff, r2)
        grad[r2 > self.comm_radius] = 0
        return grad

    def potential(self, r2):
        """:228-232 on a caller-supplied (N,N) r2: Turner potential summed over pairs."""
        p = np.reciprocal(r2) + np.log(r2)
        p[r2 > self.comm_radius2] = self.vr
        np.fill_diagonal(p, 0)
        return np.sum(np.sum(p))

    # ------------------------------------------------------------------- reset
    def _accept(self, x):
        """:177-184 on the device: min degree >= 2 and min pairwise distance >= 0.1."""
        h = self._handle()
        h.set_state(x, env=0)
        _, min_dists, deg = h.stats(0)
        return deg.min() >= 2 and min_dists.min() >= 0.1

    def reset(self):
        """:156-192."""
        x = None
        for _ in range(self.reset_max_attempts if self.reset_mode == "reference" else 1):
            x = draw_swarm(self.n_agents, self.r_max, self.v_max, self.v_bias)
            if self.reset_mode != "reference" or self._accept(x):
                break
        else:
            # the reference loops until a draw passes (flocking_relative.py:164), which
            # never ends for N >~ 200; this keeps the last draw instead, and says so
            warnings.warn("FlockingRelativeEnv.reset(): no draw met the reference's acceptance test "
                          "(min degree >= 2, min distance >= 0.1) in %d attempts; keeping the last one"
                          % self.reset_max_attempts, RuntimeWarning, stacklevel=2)
        self.mean_vel = np.mean(x[:, 2:4], axis=0)
        self.init_vel = x[:, 2:4]
        self.x = x
        self.compute_helpers()
        return (self.state_values, self.state_network)

    # ------------------------------------------------------------------ render
    def render(self, mode='human'):
        """:234-257 (matplotlib, host side)."""
        import matplotlib.pyplot as plt
        x = self.x
        if self.fig is None:
            plt.ion()
            fig = plt.figure()
            self.ax = fig.add_subplot(111)
            line1, = self.ax.plot(x[:, 0], x[:, 1], 'bo')
            self.ax.plot([0], [0], 'kx')
            plt.ylim(-1.0 * self.r_max, 1.0 * self.r_max)
            plt.xlim(-1.0 * self.r_max, 1.0 * self.r_max)
            plt.title('GNN Controller')
            self.fig, self.line1 = fig, line1
        self.line1.set_xdata(x[:, 0])
        self.line1.set_ydata(x[:, 1])
        self.fig.canvas.draw()
        self.fig.canvas.flush_events()

    def close(self):
        if self._h is not None:
            self._h.close()
            self._h = None
