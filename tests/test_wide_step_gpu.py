"""Wide envs (N = 4096, 8192: many LDS tiles, the prefetching tiled kernel) against the
CPU oracle on awkward layouts: a far outlier, a coordinate beyond any float32 band
(every pair decided in float64), 600 coincident agents plus a pile jittered below 1e-9,
all agents on one line; float32 and float64 actions; and the plain step at config 5's
full size with sampled rows (tests/test_flock_gpu.py covers config 5 with the fused
controller).

Tolerances as tests/test_flock_gpu.py: state and network bit-exact, state_values
|d| <= 1e-5 |ref| + 1e-9, reward rtol 1e-12."""
import numpy as np
import pytest

from oracle import flocking as orc

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("gym_flock._native")
from gym_flock.init_states import synthetic_batch  # noqa: E402


def check_env(h, b, x0, u, rows=None):
    xo = orc.integrate(x0, u)
    np.testing.assert_array_equal(h.get_state(b), xo)
    np.testing.assert_allclose(h.rewards()[b], orc.reward(xo), rtol=1e-12)
    n = x0.shape[0]
    if rows is None:
        ref = orc.step(x0, u)
        np.testing.assert_array_equal(h.network(b), ref["network"].astype(np.float32))
        np.testing.assert_allclose(h.state_values(b), ref["state_values"], rtol=1e-5, atol=1e-9)
    else:
        ref = orc.step_rows(x0, u, rows)
        for k, r in enumerate(rows):
            np.testing.assert_array_equal(h.network_rows(b, int(r), 1)[0], ref["network"][k].astype(np.float32))
        np.testing.assert_allclose(h.state_values(b)[rows], ref["state_values"], rtol=1e-5, atol=1e-9)
    return n


@pytest.mark.parametrize("u64", [False, True])
def test_wide_step_vs_oracle_n4096(u64):
    n, B = 4096, 3
    x0 = synthetic_batch(B, n, seed0=900)
    u = np.random.RandomState(901).uniform(-1, 1, size=(B, n, 2))
    u = u if u64 else u.astype(np.float32)
    h = nat.FlockHandle(n, B)
    h.set_state(x0)
    h.step(u)
    for b in range(B):
        check_env(h, b, x0[b], u[b])
    h.close()


def _edge_states(n):
    rs = np.random.RandomState(902)
    base = synthetic_batch(1, n, seed0=903)[0]
    far = base.copy()
    far[7, :2] = [1.0e4, -3.0e4]            # a far outlier
    huge = base.copy()
    huge[11, 0] = 5.0e13                    # past the float32 prefilter's range: float64 pairs
    pile = base.copy()
    pile[:600, :2] = pile[0, :2]            # 600 coincident agents
    pile[600:900, :2] = pile[600, :2] + rs.uniform(-1e-9, 1e-9, size=(300, 2))
    line = base.copy()
    line[:, 1] = 0.0                        # all agents on a line
    line[:, 0] = np.linspace(-50, 50, n)
    return {"far": far, "huge": huge, "pile": pile, "line": line}


@pytest.mark.parametrize("case", ["far", "huge", "pile", "line"])
def test_wide_step_edge_layouts(case):
    n = 4096
    x0 = _edge_states(n)[case]
    u = np.random.RandomState(904).uniform(-1, 1, size=(1, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, 1)
    h.set_state(x0[None])
    h.step(u)
    xo = orc.integrate(x0, u[0])
    np.testing.assert_array_equal(h.get_state(0), xo)
    ref = orc.step(x0, u[0])
    np.testing.assert_array_equal(h.network(0), ref["network"].astype(np.float32))
    np.testing.assert_allclose(h.state_values(0), ref["state_values"], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(h.rewards()[0], ref["reward"], rtol=1e-12)
    h.close()


def test_plain_step_config5_sampled_oracle():
    """BASELINE.json configs[4] (32 envs x N=8192), the bench's plain step: every env's
    state bit-exact and reward (rtol 1e-12); sampled rows of 3 envs against the oracle."""
    n, B = 8192, 32
    x0 = synthetic_batch(B, n, seed0=907)
    u = np.random.RandomState(908).uniform(-1, 1, size=(B, n, 2)).astype(np.float32)
    h = nat.FlockHandle(n, B)
    h.set_state(x0)
    h.step(u)
    x1, rew = h.get_state(), h.rewards()
    for b in range(B):
        xo = orc.integrate(x0[b], u[b])
        np.testing.assert_array_equal(x1[b], xo)
        np.testing.assert_allclose(rew[b], orc.reward(xo), rtol=1e-12)
    rs = np.random.RandomState(909)
    for b in (0, 17, 31):
        rows = np.unique(np.concatenate([[0, 15, 16, 4095, 8191], rs.choice(n, 19, replace=False)]))
        check_env(h, b, x0[b], u[b], rows)
    h.close()
