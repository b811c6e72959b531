"""Stream-ordering contracts of a split-step handle (two half-batch launches per step on
two HIP streams), exercised through the raw HIP runtime the library itself is bound to
(ctypes on the libamdhip64 already mapped into the process; no torch):

* after fe_sync, a zero-copy consumer may enqueue reads of the outputs on the handle's
  stream (fe_buffers.stream); the next step's second half must not overwrite them first;
* device-resident actions (FE_U_DEVICE) written by the caller on the handle's stream
  before each step give the same bits with split steps as with one launch per step.
"""
import ctypes

import numpy as np
import pytest

from gym_flock import _native as nat
from gym_flock.init_states import synthetic_batch

pytestmark = pytest.mark.gpu

H2D, D2H, D2D = 1, 2, 3


def hip_runtime():
    nat.load()
    with open("/proc/self/maps") as f:
        paths = {ln.split()[-1] for ln in f if "libamdhip64.so" in ln}
    assert paths, "libamdhip64 is not mapped after loading libgymflock"
    hip = ctypes.CDLL(sorted(paths)[0])
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipDeviceSynchronize.argtypes = []
    return hip


def hmalloc(hip, n):
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), n) == 0
    return p.value


def test_consumer_reads_after_sync_precede_next_split_step():
    hip = hip_runtime()
    B, N = 8, 1024
    h = nat.FlockHandle(N, B)
    h.set_state(synthetic_batch(B, N, seed0=4100))
    h.set_actions(np.random.RandomState(4101).uniform(-1, 1, size=(B, N, 2)).astype(np.float32))
    for _ in range(2):
        h.step(None, nat.FE_U_RESIDENT)
    want = h.network()
    h.sync()
    buf = h.device_buffers()
    nbytes = B * N * N * 4
    big = 1 << 30  # a 1 GiB device copy ahead of the consumer's read keeps `stream` busy
    a, b, snap = hmalloc(hip, big), hmalloc(hip, big), hmalloc(hip, nbytes)
    try:
        assert hip.hipMemcpyAsync(b, a, big, D2D, buf.stream) == 0
        assert hip.hipMemcpyAsync(snap, buf.network, nbytes, D2D, buf.stream) == 0
        h.step(None, nat.FE_U_RESIDENT)  # split: the second half must wait for the reads
        h.sync()
        got = np.empty((B, N, N), np.float32)
        assert hip.hipMemcpy(got.ctypes.data, snap, nbytes, D2H) == 0
    finally:
        for p in (a, b, snap):
            hip.hipFree(p)
        h.close()
    np.testing.assert_array_equal(got, want)


def test_device_actions_split_match_single_stream():
    hip = hip_runtime()
    B, N, steps = 5, 300, 6
    x0 = synthetic_batch(B, N, seed0=4200)
    rs = np.random.RandomState(4201)
    us = [rs.uniform(-1, 1, size=(B, N, 2)).astype(np.float32) for _ in range(steps)]
    outs = []
    for streams in (2, 1):
        h = nat.FlockHandle(N, B)
        h.set_streams(streams)
        h.set_state(x0)
        stream = h.device_buffers().stream
        du = [hmalloc(hip, us[0].nbytes) for _ in range(steps)]
        try:
            got = []
            for t in range(steps):
                # the caller writes this step's actions on the handle's stream, then steps
                # (a buffer per step: earlier steps' second halves may still read theirs)
                assert hip.hipMemcpyAsync(du[t], us[t].ctypes.data, us[t].nbytes, H2D, stream) == 0
                h.step(du[t], nat.FE_U_DEVICE)
                if t % 3 == 2:
                    got += [h.get_state(), h.network(), h.rewards()]
            outs.append(got)
        finally:
            h.sync()
            for p in du:
                hip.hipFree(p)
            h.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
    # and the same bits as host actions
    h = nat.FlockHandle(N, B)
    h.set_state(x0)
    for t in range(steps):
        h.step(us[t])
    np.testing.assert_array_equal(h.get_state(), outs[0][-3])
    h.close()


@pytest.mark.parametrize("f64", [False, True])
def test_host_actions_pipelined_split_steps(f64):
    """Host actions of split steps go through the action stream into two device buffers,
    so each copy overlaps the step before. 16 back-to-back steps, each call given the same
    numpy array overwritten right after it returns (the call must have copied it by then),
    with resident-action steps and a getter mixed in: every state and reward bit-exact
    against one-launch steps on a second handle with the actions set per step, and
    against the oracle for two envs."""
    from oracle import flocking as orc
    B, N, T = 6, 256, 16
    x0 = synthetic_batch(B, N, seed0=77)
    us = np.random.RandomState(5).uniform(-1, 1, size=(T, B, N, 2)).astype(np.float64 if f64 else np.float32)
    flags = nat.FE_U_F64 if f64 else 0
    h = nat.FlockHandle(N, B)
    g = nat.FlockHandle(N, B)
    g.set_streams(1)
    h.set_state(x0)
    g.set_state(x0)
    buf = np.empty_like(us[0])
    rew_h, rew_g = [], []
    for t in range(T):
        if t == 9:
            h.set_actions(us[t])
            h.step(None, nat.FE_U_RESIDENT | flags)
        else:
            buf[...] = us[t]
            h.step(buf, flags)
            buf[...] = np.nan  # the borrowed array is free again once the call returned
        g.set_actions(us[t])
        g.step(None, nat.FE_U_RESIDENT | flags)
        if t % 5 == 4:  # (a getter: the step after it is one launch, the others split)
            np.testing.assert_array_equal(h.get_state(), g.get_state())
            rew_h.append(h.rewards())
            rew_g.append(g.rewards())
    np.testing.assert_array_equal(h.get_state(), g.get_state())
    np.testing.assert_array_equal(np.array(rew_h), np.array(rew_g))
    for b in (0, B - 1):
        x = x0[b]
        for t in range(T):
            x = orc.integrate(x, us[t, b])
        np.testing.assert_array_equal(h.get_state(b), x)
    h.close()
    g.close()
