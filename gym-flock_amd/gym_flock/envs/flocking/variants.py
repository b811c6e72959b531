"""The registered flocking variants on the MI355X engine: drop-ins for the reference's
gym_flock/envs/flocking/flocking_{leader,obstacle,stoch,twoflocks}.py.

Each is a FlockingRelativeEnv whose step runs on the same fused kernel with the
fe_variant switches of include/gymflock.h. The switches are:
  - the step's action scale;
  - a prefix of frozen agents (their mask is 0);
  - zeroed velocity differences for pairs that touch the first agents;
  - action and controller clips;
  - the stochastic env's state scale and per-step dt.
Host code keeps what the reference draws from the global np.random (resets, the
stochastic dt) in the reference's call order. Seeded runs therefore reproduce the
reference episodes (tests/golden/variant_*.npz).
"""
import numpy as np

from .flocking_relative import FlockingRelativeEnv


def grid(N, side=5):
    """utils.py:26-33 (flocking_obstacle.py:4-11 has the same helper)."""
    side2 = int(N / side)
    xs = np.arange(0, side) - side / 2.0
    ys = np.arange(0, side2) - side2 / 2.0
    xs, ys = np.meshgrid(xs, ys)
    xs = xs.reshape((N, 1))
    ys = ys.reshape((N, 1))
    return 0.8 * np.hstack((xs, ys))


def _frozen_prefix(mask, n_agents, strict=False):
    """Number of leading zeros of a 0/1 mask that is zero on a prefix only (the only
    shape the reference builds). With strict, a mask sized for another agent count
    fails the way NumPy broadcasting fails in the reference step (:41-49)."""
    mask = np.asarray(mask)
    if mask.shape != (n_agents,):
        if strict:
            raise ValueError("operands could not be broadcast together with shapes (%d,) (%d,)"
                             % (n_agents, mask.shape[0]))
        mask = mask[:n_agents]
    nz = np.flatnonzero(mask == 0)
    k = len(nz)
    if not (np.array_equal(nz, np.arange(k)) and np.all(mask[k:] == 1)):
        raise NotImplementedError("only masks that freeze a prefix of agents are supported")
    return k


class FlockingLeaderEnv(FlockingRelativeEnv):
    """flocking_leader.py: two leaders that ignore actions. The step leaves actions
    unscaled (:21-33). reset() gives the leaders one shared random velocity after the
    relative reset (:37-41)."""

    def __init__(self, device=0):
        super(FlockingLeaderEnv, self).__init__(device)
        self.n_leaders = 2
        self.mask = np.ones((self.n_agents,))
        self.mask[0:self.n_leaders] = 0
        self.quiver = None
        self.half_leaders = int(self.n_leaders / 2.0)

    def params_from_cfg(self, args):
        super(FlockingLeaderEnv, self).params_from_cfg(args)
        self.mask = np.ones((self.n_agents,))
        self.mask[0:self.n_leaders] = 0

    def _variant(self):
        return dict(u_scale=1.0, n_frozen=_frozen_prefix(self.mask, self.n_agents))

    def step(self, u):
        u = np.asarray(u)
        assert u.shape == (self.n_agents, self.nu)
        _frozen_prefix(self.mask, self.n_agents, strict=True)
        self.u = u
        self._helpers_x = None
        self._device_step(u)
        return (self.state_values, self.state_network), self._reward, False, {}

    def reset(self):
        obs = super(FlockingLeaderEnv, self).reset()
        x = self.x
        self._helpers_x = x.copy()  # the state compute_helpers last saw
        x[0:self.n_leaders, 2:4] = np.ones((self.n_leaders, 2)) * np.random.uniform(
            low=-self.v_max, high=self.v_max, size=(1, 1))
        self.x = x
        h = self._handle()
        h.compute_helpers()  # instant_cost() reads the current x in the reference
        self._reward = float(h.rewards()[0])
        return obs  # the reference returns the observation computed before the override

    def controller(self, centralized=None):
        """Until the next step the reference's controller still sees the diff that
        reset() computed before the leader override (flocking_leader.py:37-41 sets x
        after compute_helpers); the device evaluates it on that state."""
        before = getattr(self, "_helpers_x", None)
        if before is None:
            return super(FlockingLeaderEnv, self).controller(centralized)
        h = self._handle()
        now = self.x
        h.set_state(before, env=0)
        try:
            return super(FlockingLeaderEnv, self).controller(centralized)
        finally:
            h.set_state(now, env=0)


class FlockingObstacleEnv(FlockingRelativeEnv):
    """flocking_obstacle.py: four static obstacles. They ignore actions (:34-49), and
    no velocity difference is counted for any pair that touches them (:75-80). The
    reset is a deterministic grid (:59-74)."""

    def __init__(self, device=0):
        super(FlockingObstacleEnv, self).__init__(device)
        self.n_obstacles = 4
        self.mask = np.ones((self.n_agents,))
        self.mask[0:self.n_obstacles] = 0
        self.r_max = 3.0
        self.line1 = None
        self.line2 = None

    def params_from_cfg(self, args):
        # like the reference, the mask keeps the size it got in __init__ (:25-27)
        super(FlockingObstacleEnv, self).params_from_cfg(args)
        self.mask[0:self.n_obstacles] = 0

    def _variant(self):
        return dict(u_scale=1.0, n_frozen=_frozen_prefix(self.mask, self.n_agents),
                    n_vel_zero=self.n_obstacles)

    def step(self, u):
        u = np.asarray(u)
        assert u.shape == (self.n_agents, self.nu)
        _frozen_prefix(self.mask, self.n_agents, strict=True)
        self.u = u
        self._device_step(u)
        return (self.state_values, self.state_network), self._reward, False, {}

    def reset(self):
        x = np.zeros((self.n_agents, self.nx_system))
        x[:, 0:2] = grid(self.n_agents)
        x[:, 2:4] = [0, -7.0]
        x[0:self.n_obstacles, 0:2] = grid(self.n_obstacles, side=2) * 0.5
        x[0:self.n_obstacles, 1] -= 10.0
        x[0:self.n_obstacles, 2:4] = 0
        self.mean_vel = np.mean(x[self.n_obstacles:, 2:4], axis=0)
        self.init_vel = x[self.n_obstacles:, 2:4]
        self.x = x
        self.compute_helpers()
        return (self.state_values, self.state_network)

    def render(self, mode='human'):
        super(FlockingObstacleEnv, self).render(mode)
        x = self.x
        if self.line2 is None:
            self.line2, = self.ax.plot(x[:self.n_obstacles, 0], x[:self.n_obstacles, 1], 'ro')
        self.line2.set_xdata(x[:self.n_obstacles, 0])
        self.line2.set_ydata(x[:self.n_obstacles, 1])
        self.fig.canvas.draw()
        self.fig.canvas.flush_events()


class FlockingStochasticEnv(FlockingRelativeEnv):
    """flocking_stoch.py. Actions are clipped to +-0.5 and scaled by 6, and the state
    is scaled by 6 around the update (:14-36). dt ~ N(0.12, 0.018) is drawn from the
    global RNG on every step (:24). The expert is clipped to +-0.5 (:39-46)."""

    def __init__(self, device=0):
        super(FlockingStochasticEnv, self).__init__(device)
        self.dt_mean = 0.12
        self.dt_sigma = 0.018
        self.max_accel = 0.5
        self.scale = 6.0

    def _key_dt(self):
        return self.dt_mean  # dt changes every step; it goes to the device per step (fe_set_dt)

    def _variant(self):
        return dict(u_scale=self.scale, u_clip=self.max_accel, x_scale=self.scale,
                    ctrl_clip=self.max_accel)

    def step(self, u):
        u = np.asarray(u)
        assert u.shape == (self.n_agents, self.nu)
        u = np.clip(u, a_min=-self.max_accel, a_max=self.max_accel)
        self.u = u * self.scale
        self.dt = np.random.normal(self.dt_mean, self.dt_sigma)
        self._handle().set_dt(self.dt)
        self._device_step(u)
        return (self.state_values, self.state_network), self._reward, False, {}


class FlockingTwoFlocksEnv(FlockingRelativeEnv):
    """flocking_twoflocks.py. Only the reset differs (:8-28): agents start on a grid
    with velocities opposite to their positions, plus one global-RNG bias."""

    def reset(self):
        x = np.zeros((self.n_agents, self.nx_system))
        bias = np.random.uniform(low=-self.v_bias / 2.0, high=self.v_bias / 2.0, size=(2,))
        grids = grid(self.n_agents, side=int(self.n_agents / 10))
        x[:, 0:2] = grids
        x[:, 2:4] = -grids
        x[:, 2] = x[:, 2] + bias[0]
        x[:, 3] = x[:, 3] + bias[1]
        self.mean_vel = np.mean(x[:, 2:4], axis=0)
        self.init_vel = x[:, 2:4]
        self.x = x
        self.compute_helpers()
        return (self.state_values, self.state_network)
