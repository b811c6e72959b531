"""World-size-2 gloo test of the multi-GPU path's logic on CPU: each rank owns a
contiguous shard of the env batch (shard_range), computes its envs' rewards (here
with the oracle, since there is no GPU) and all-gathers them (GlooRewardGather);
the gathered vector must equal the single-process batch in global env order."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

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


def _worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
    import torch.distributed as dist
    from gym_flock.shard import GlooRewardGather, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, stop = shard_range(TOTAL_ENVS, world, rank)
    got = GlooRewardGather().gather(_rewards_for(start, stop))
    if rank == 0:
        q.put(got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_sharded_reward_allgather_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(got, _rewards_for(0, TOTAL_ENVS))
