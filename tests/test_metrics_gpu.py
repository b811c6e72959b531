"""The RCCL metrics path (include/gymflock.h fe_comm_* / fe_allgather_*)
on one GPU: the reward all-gather ships every step since the previous gather exactly
once at any interval, refuses a gap longer than the ring; a communicator whose peers
never join fails within its timeout and leaves the handle stepping; RCCL's own view of
the communicator; destroy and re-init. Multi-rank layouts (uneven shards padded to the
largest) are covered on the CPU (test_shard_gloo, test_capi_cpu)."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from conftest import ROOT
from oracle import flocking as orc

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("gym_flock._native")
from gym_flock.init_states import synthetic_batch  # noqa: E402
from gym_flock.shard import RcclRewardGather  # noqa: E402
from gym_flock.vec import VecFlockingRelative  # noqa: E402


@pytest.mark.parametrize("interval", [3, 5, 8, 13])
def test_reward_gather_every_step_once(interval):
    """Gathers every `interval` steps over 70 steps (the 64-slot ring wraps): the
    concatenated gathered rows equal the rewards of every step, in order, each once."""
    B, N = 4, 64
    v = VecFlockingRelative(B, N)
    v.reset(seed=3)
    g = RcclRewardGather(v.h, 1, 0, v.h.comm_unique_id(), timeout=60.0)
    u = np.random.RandomState(0).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    hist, got = [], []
    for t in range(70):
        v.step(u)
        hist.append(v.rewards())
        if (t + 1) % interval == 0:
            g.issue()
            got.append(g.result())
            assert got[-1].shape == (interval, B)
    if len(hist) % interval:
        g.issue()
        got.append(g.result())
    np.testing.assert_array_equal(np.concatenate(got), np.array(hist))
    with pytest.raises(nat.GymFlockError) as e:  # nothing new to ship
        g.issue()
    assert e.value.code == nat.GF_ESTATE
    v.close()


def test_reward_gather_gap_longer_than_ring():
    """More than 64 steps between gathers: the oldest rewards were overwritten, so the
    gather refuses (GF_ESTATE) and skips them; the next gather ships the next steps."""
    B, N = 3, 32
    v = VecFlockingRelative(B, N)
    v.reset(seed=1)
    g = RcclRewardGather(v.h, 1, 0, v.h.comm_unique_id(), timeout=60.0)
    u = np.random.RandomState(1).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    for _ in range(65):
        v.step(u)
    with pytest.raises(nat.GymFlockError) as e:
        g.issue()
    assert e.value.code == nat.GF_ESTATE and "overwritten" in str(e.value)
    want = []
    for _ in range(2):
        v.step(u)
        want.append(v.rewards())
    g.issue()
    np.testing.assert_array_equal(g.result(), np.array(want))
    v.close()


def test_comm_info_destroy_reinit():
    """RCCL's own view at one rank (count 1, user rank 0, device 0 and its PCI bus id);
    fe_comm_destroy tears the metrics path down and a second init works."""
    B, N = 2, 32
    h = nat.FlockHandle(N, B)
    h.set_state(synthetic_batch(B, N))
    u = np.zeros((B, N, 2), np.float32)
    for rnd in range(2):
        h.comm_init(1, 0, nat.FlockHandle.comm_unique_id(), timeout=60.0)
        info = h.comm_info()
        assert info["count"] == 1 and info["user_rank"] == 0 and info["device"] == 0
        assert len(info["pci_bus_id"]) >= 7, info
        assert h.shard_sizes == [B] and h.max_envs == B
        h.step(u, 0)
        h.allgather_rewards()
        np.testing.assert_array_equal(h.gathered_rewards()[0, -1], h.rewards())
        h.comm_destroy()
        with pytest.raises(nat.GymFlockError) as e:
            h.allgather_rewards()
        assert e.value.code == nat.GF_ESTATE
    h.close()


_LONE_RANK = r"""
import sys, time
import numpy as np
sys.path[:0] = [{root!r}, {pkg!r}]
from gym_flock import _native as nat
from gym_flock.init_states import synthetic_batch
from oracle import flocking as orc
B, N = 2, 48
h = nat.FlockHandle(N, B)
x0 = synthetic_batch(B, N, seed0=4)
h.set_state(x0)
t0 = time.monotonic()
try:
    h.comm_init(2, 0, nat.FlockHandle.comm_unique_id(), timeout=5.0)
    print("INIT_OK")
except nat.GymFlockError as e:
    print("CODE", e.code, "SECONDS", round(time.monotonic() - t0, 2))
    print("MSG", str(e).replace("\n", " "))
u = np.random.RandomState(2).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
h.step(u, 0)
x1 = h.get_state()
ok = all(np.array_equal(x1[b], orc.step(x0[b], u[b])["x"]) for b in range(B))
print("STEP_OK", ok)
h.close()
"""


def test_comm_init_peer_never_joins():
    """Rank 0 of a 2-rank communicator whose rank 1 never starts: fe_comm_init_timeout
    (5 s) returns GF_ECOMM within 15 s (non-blocking init polled, then aborted) and the
    handle still steps, bit-exact against the oracle. In a child process, so a hang
    there cannot take the test runner with it."""
    code = _LONE_RANK.format(root=ROOT, pkg=os.path.join(ROOT, "gym-flock_amd"))
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=90)
    wall = time.monotonic() - t0
    out = p.stdout.decode()
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    assert "INIT_OK" not in out
    fields = dict(ln.split(" ", 1) for ln in out.splitlines() if " " in ln)
    code_s, secs = fields["CODE"].split(" SECONDS ")
    assert int(code_s) == nat.GF_ECOMM, out
    assert float(secs) < 15.0, out
    assert "timed out" in fields["MSG"], out
    assert fields["STEP_OK"] == "True", out
    print("lone-rank init failed after %s s (child wall %.1f s): %s" % (secs, wall, fields["MSG"]))


def test_steps_never_wait_behind_a_stuck_collective():
    """A collective that does not complete (a gate kernel holds the collectives' side
    stream, as a peer that stopped responding would) does not hold the step streams: they
    never wait on the side stream on the device. 56 steps (and their reward reads) after
    a gather queued behind the gate finish while it is shut. The step that reuses that
    gather's first ring slot (64 steps on) waits for its staging copy on the host, bounded
    by the collective timeout, and goes on as soon as the gate opens (2 s later here); the
    gather then delivers exactly its steps."""
    import threading
    B, N = 3, 32
    v = VecFlockingRelative(B, N)
    v.reset(seed=5)
    g = RcclRewardGather(v.h, 1, 0, v.h.comm_unique_id(), timeout=60.0)
    u = np.random.RandomState(5).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
    for _ in range(8):  # steps 0-7
        v.step(u)
    g.issue()
    g.result()
    v.h.debug_comm_gate(True, max_seconds=30.0)
    opener = None
    try:
        t_gate = time.monotonic()  # the gate kernel runs before anything is queued behind it
        while v.h.debug_comm_state()["gate_started"] != 1 and time.monotonic() - t_gate < 10.0:
            time.sleep(0.001)
        st_gate = v.h.debug_comm_state()
        hist = []
        for _ in range(8):  # steps 8-15
            v.step(u)
            hist.append(v.rewards())
        g.issue()  # its staging copy and collective queue behind the gate
        st_issue = v.h.debug_comm_state()
        t0 = time.monotonic()
        for _ in range(56):  # steps 16-71: no ring slot of the pending gather is reused
            v.step(u)
            v.rewards()
        free_run = time.monotonic() - t0
        opener = threading.Timer(2.0, lambda: v.h.debug_comm_gate(False))
        opener.start()
        t1 = time.monotonic()
        v.step(u)  # step 72 reuses step 8's slot: waits (host, bounded) for the staging copy
        v.rewards()
        waited = time.monotonic() - t1
        st_reuse = v.h.debug_comm_state()
    finally:
        if opener is not None:
            opener.join()
        v.h.debug_comm_gate(False)
    print("gate:", st_gate, "\nissue:", st_issue, "\nreuse:", st_reuse, "\nwaited %.3f s" % waited)
    assert st_gate["gate_started"] == 1 and st_gate["gate_ended"] == 0, st_gate
    assert st_issue["gather_copy_done"] == 0, st_issue     # queued behind the gate
    assert st_reuse["reuse_copy_done"] == 0, st_reuse      # still behind it 56 steps on
    assert st_reuse["reuse_wait_rc"] == 0 and st_reuse["comm_live"] == 1, st_reuse
    assert st_reuse["gate_ended"] == 1, st_reuse
    assert free_run < 5.0, "steps waited %.1f s behind the gated collective" % free_run
    assert 1.0 < waited < 15.0, waited
    np.testing.assert_array_equal(g.result(), np.array(hist))
    v.close()


_ABORT_MID_RUN = r"""
import sys, time
import numpy as np
sys.path[:0] = [{root!r}, {pkg!r}]
from gym_flock import _native as nat
from gym_flock.vec import VecFlockingRelative
from gym_flock.shard import RcclRewardGather
B, N = 3, 32
v = VecFlockingRelative(B, N)
v.reset(seed=5)
g = RcclRewardGather(v.h, 1, 0, v.h.comm_unique_id(), timeout=3.0)
u = np.random.RandomState(5).uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
for _ in range(8):
    v.step(u)
g.issue()
print("FIRST_OK", g.result().shape)
v.h.debug_comm_gate(True, max_seconds=25.0)
try:
    for _ in range(4):
        v.step(u)
    g.issue()  # queued behind the gate: it never completes within the timeout
    t0 = time.monotonic()
    try:
        g.result()
        print("RESULT_OK")
    except nat.GymFlockError as e:
        print("CODE", e.code, "SECONDS", round(time.monotonic() - t0, 2))
        print("MSG", str(e).replace("\n", " "))
    t1 = time.monotonic()
    for _ in range(10):  # the handle keeps stepping, its rewards stay readable
        v.step(u)
        r = v.rewards()
    print("STEPS_SECONDS", round(time.monotonic() - t1, 2), "STEP_OK", bool(np.isfinite(r[0]).all()))
    try:
        g.issue()
        print("REISSUE_OK")
    except nat.GymFlockError as e:
        print("REISSUE", e.code, str(e).replace("\n", " "))
finally:
    v.h.debug_comm_gate(False)
v.sync()
v.close()
print("DONE")
"""


def test_collective_timeout_aborts_mid_run():
    """The mid-run abort path (comm_event_wait): a reward gather whose collective never
    completes (queued behind the gate kernel on the side stream, as behind a dead peer)
    fails with GF_ECOMM after the collective timeout (3 s here), the communicator is
    aborted on the process's communicator worker, the handle keeps stepping with its
    rewards readable, and the metrics path then reports why it is gone (GF_ESTATE). In a
    child process (a fresh HIP context; the gate is released before it exits)."""
    code = _ABORT_MID_RUN.format(root=ROOT, pkg=os.path.join(ROOT, "gym-flock_amd"))
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=120)
    wall = time.monotonic() - t0
    out = p.stdout.decode(errors="replace") + p.stderr.decode(errors="replace")
    assert p.returncode == 0, out
    fields = {}
    for line in p.stdout.decode().splitlines():
        k, _, rest = line.partition(" ")
        fields[k] = rest
    assert "FIRST_OK" in fields and "DONE" in fields, out
    code_s, _, secs = fields["CODE"].partition(" SECONDS ")
    assert int(code_s) == nat.GF_ECOMM, out
    assert 2.5 < float(secs) < 15.0, out
    assert "aborted" in fields["MSG"], out
    steps_s, _, ok = fields["STEPS_SECONDS"].partition(" STEP_OK ")
    assert ok == "True" and float(steps_s) < 5.0, out
    assert fields["REISSUE"].split()[0] == str(nat.GF_ESTATE), out
    assert "timed out" in fields["REISSUE"], out  # the reason the metrics path is gone
    print("collective timed out after %s s, communicator aborted (child wall %.1f s)" % (secs, wall))
