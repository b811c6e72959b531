"""World-size-2 CPU test of the multi-rank bench's host side, without torch: the
HostGroup rendezvous from torchrun's environment variables (HostGroup.from_env), the
broadcast of rank 0's 128-byte RCCL unique id, barriers, the max over ranks, and
check_gathered(), with which every rank verifies the WHOLE gathered reward vector
against the ranks' local rewards. The RCCL all-gather itself needs GPUs; here the
gathered vector comes from the host channel (HostRewardGather), and one run corrupts
one element of rank 1's copy to show that every rank then reports the failure."""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

from conftest import ROOT

TOTAL_ENVS, N = 5, 32


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rewards_for(start, stop):
    from gym_flock.init_states import synthetic_state
    from oracle import flocking as orc
    out = []
    for g in range(start, stop):
        x = synthetic_state(N, g)
        u = np.random.RandomState(10_000 + g).uniform(-1, 1, size=(N, 2)).astype(np.float32)
        out.append(orc.step(x, u)["reward"])
    return np.array(out)


def _worker(rank, world, port, corrupt, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port - 1))
    from gym_flock.hostgroup import HostGroup
    from gym_flock.shard import HostRewardGather, check_gathered, shard_range
    with HostGroup.from_env(timeout=60) as g:
        uid = g.broadcast_bytes(os.urandom(128) if rank == 0 else b"")
        start, stop = shard_range(TOTAL_ENVS, world, rank)
        local = _rewards_for(start, stop)
        g.barrier()
        gathered = HostRewardGather(g).gather(local)
        if corrupt and rank == 1:
            gathered = gathered.copy()
            gathered[0] += 1e-9
        mine, every = check_gathered(g, gathered, local)
        tmax = g.max(0.5 + rank)
        q.put((rank, uid, gathered, mine, every, tmax, "torch" in sys.modules))


@pytest.mark.timeout(120)
@pytest.mark.parametrize("corrupt", [False, True])
def test_two_ranks_rendezvous_and_whole_vector_check(corrupt):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, corrupt, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, uid0, g0, m0, e0, t0, torch0), (r1, uid1, g1, m1, e1, t1, torch1) = res
    assert uid0 == uid1 and len(uid0) == 128
    assert t0 == t1 == 1.5
    assert not torch0 and not torch1  # the host side never imports torch
    np.testing.assert_array_equal(g0, _rewards_for(0, TOTAL_ENVS))
    if corrupt:
        assert m0 and not m1 and not e0 and not e1
    else:
        assert m0 and m1 and e0 and e1


@pytest.mark.timeout(180)
def test_eight_ranks_rendezvous_and_whole_vector_check():
    """The driver's 8-GPU shape (one rank per GPU) on the CPU: 8 ranks meet over the host
    channel, share rank 0's unique id, agree on the max time, and each verifies the whole
    gathered vector (5 envs over 8 ranks: some ranks hold none)."""
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, False, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=150) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _rewards_for(0, TOTAL_ENVS)
    for rank, uid, gathered, mine, every, tmax, imported_torch in res:
        assert uid == res[0][1] and len(uid) == 128
        assert tmax == world - 0.5
        assert mine and every and not imported_torch
        np.testing.assert_array_equal(gathered, want)


@pytest.mark.timeout(60)
def test_rendezvous_drops_stray_peers_and_goes_on():
    """Processes that reach rank 0's port during the rendezvous with the wrong token, or
    that connect and send nothing, are dropped (bench.py's launcher sets
    GYMFLOCK_HOST_TOKEN; nothing received is ever unpickled), and the real rank 1 still
    joins; with rank 1 missing, rank 0 fails at the timeout with its peers closed."""
    import struct
    import threading
    import time
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
    from gym_flock.hostgroup import HostGroup
    port = _free_port()
    out, err = [], []

    def rank0(timeout):
        try:
            g = HostGroup(0, 2, "127.0.0.1", port, timeout=timeout, token=b"k" * 32)
            out.append(g)
        except Exception as e:  # noqa: BLE001
            err.append(e)

    def connect():
        for _ in range(200):
            try:
                return socket.create_connection(("127.0.0.1", port), timeout=5)
            except OSError:
                time.sleep(0.05)
        raise AssertionError("rank 0 never listened")

    HostGroup.HELLO_TIMEOUT = 1.0
    t = threading.Thread(target=rank0, args=(30,))
    t.start()
    bad = connect()
    bad.sendall(struct.pack("!I", 1) + b"x" * 32)   # wrong token
    silent = connect()                                # says nothing
    g1 = HostGroup(1, 2, "127.0.0.1", port, timeout=30, token=b"k" * 32)
    t.join(timeout=40)
    bad.close()
    silent.close()
    assert not err and out, err
    g0 = out[0]
    assert len(g0.refused) == 2
    done1 = []
    t1 = threading.Thread(target=lambda: done1.append(g1.barrier() is None))
    t1.start()
    g0.barrier()
    t1.join(timeout=30)   # rank 1's barrier returned before either side closes
    assert not t1.is_alive() and done1 == [True], done1
    g0.close()
    g1.close()

    # nobody joins: a bounded failure, not a hang
    port = _free_port()
    t0 = time.monotonic()
    rank0(2)
    assert err and "ranks joined" in str(err[-1]) and time.monotonic() - t0 < 10


def test_struct_messages_only():
    """The group's typed gathers are fixed-format struct values (no pickle anywhere)."""
    src = open(os.path.join(ROOT, "gym-flock_amd", "gym_flock", "hostgroup.py")).read()
    assert "import pickle" not in src and "pickle.loads" not in src and "eval(" not in src
