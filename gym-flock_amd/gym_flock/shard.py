"""Multi-GPU sharding of the env batch.

Envs are independent, so the batch is split into contiguous ranges, one per rank
(one process per GPU); the step path has no exchange. The only collective is the
metrics path: per-env rewards are all-gathered so every rank (or the trainer on
rank 0) sees the whole batch's rewards in global env order; optionally the per-env
get_stats summaries (means of vel_diffs and min_dists) likewise.

Transports for that all-gather:
  - RcclRewardGather: RCCL over xGMI, issued by libgymflock on a side stream right
    after the step kernel (fe_allgather_rewards) — the GPU path.
  - HostRewardGather: the torch-free host channel (hostgroup.HostGroup) on host
    copies — the CPU tests and CPU-only callers.
  - GlooRewardGather: torch.distributed (gloo) on host copies — for callers that
    already hold a gloo group.
check_gathered() is how every rank verifies the WHOLE gathered vector against the
ranks' local rewards, exchanged over the host channel. torch is imported lazily and
only by the gloo transport: the env and the multi-rank bench have no PyTorch
dependency.
"""
import numpy as np


def shard_range(total_envs, world_size, rank):
    """Contiguous [start, stop) of global env indices owned by `rank`; the first
    total_envs % world_size ranks hold one extra env."""
    if not (0 <= rank < world_size):
        raise ValueError("rank out of range")
    q, r = divmod(int(total_envs), int(world_size))
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


class RcclRewardGather:
    """All-gather of per-env rewards with RCCL (equal shard sizes on every rank).

    issue() after a step enqueues one collective for the steps since the start of the
    current 8-step block (call it every 8 steps to ship each step's rewards once);
    result() returns them as (steps, world * B) in global env order."""

    def __init__(self, handle, world_size, rank, unique_id, timeout=300.0):
        self.handle = handle
        handle.comm_init(world_size, rank, unique_id, timeout)

    def issue(self):
        self.handle.allgather_rewards()

    def result(self):
        g = self.handle.gathered_rewards()  # (world, steps, B)
        return np.concatenate(list(g), axis=1)

    def issue_stats(self):
        """The optional get_stats aggregates: every rank's per-env means of
        vel_diffs and min_dists of the current state, all-gathered on the side stream."""
        self.handle.allgather_stats()

    def stats_result(self):
        """(world * B, 2) per-env [mean vel_diffs, mean min_dists] in global env order."""
        return self.handle.gathered_stats().reshape(-1, 2)


def check_equal_shards(group, n_envs):
    """Every rank's env count over the host channel; raises on every rank unless they are
    equal (the RCCL reward all-gather ships one count per rank; fe_comm_init checks the
    same on the device). Returns the per-rank counts."""
    sizes = group.allgather_i64(int(n_envs))
    if len(set(sizes)) != 1:
        raise RuntimeError("unequal env shards over ranks: n_envs per rank = %s (the reward all-gather "
                           "needs the same count on every rank)" % sizes)
    return sizes


def init_rccl_gather(group, handle, world, rank, timeout=300.0):
    """The multi-rank path's RCCL setup, bounded by the host channel: the ranks' shard
    sizes are compared first; rank 0's unique id goes out only once every rank has joined
    the channel (HostGroup's rendezvous); each rank's bounded communicator init
    (fe_comm_init_timeout) reports success over the channel, and every rank raises if any
    rank failed, instead of leaving the others in RCCL. Returns an RcclRewardGather."""
    check_equal_shards(group, handle.n_envs)
    uid = group.broadcast_bytes(handle.comm_unique_id() if rank == 0 else b"")
    err = None
    try:
        gather = RcclRewardGather(handle, world, rank, uid, timeout)
    except Exception as e:  # reported to every rank below, then re-raised here
        err, gather = e, None
    ok = group.allgather_bool(err is None)
    if err is not None:
        raise err
    if not all(ok):
        raise RuntimeError("RCCL communicator init failed on rank(s) %s" % [r for r, v in enumerate(ok) if not v])
    return gather


class HostRewardGather:
    """All-gather of per-env rewards over a HostGroup (host copies, any shard sizes)."""

    def __init__(self, group):
        self.group = group

    def gather(self, local_rewards):
        parts = self.group.allgather_bytes(np.ascontiguousarray(local_rewards, dtype=np.float64).tobytes())
        return np.concatenate([np.frombuffer(p, np.float64) for p in parts])


def check_gathered(group, gathered, local_rewards):
    """Every rank checks the whole gathered (world * B,) reward vector (or any per-env
    float64 array, e.g. the (world * B, 2) stats summaries) against the ranks' local
    values, sent over the host channel and concatenated in rank order. Returns (this
    rank's check, every rank's check)."""
    want = HostRewardGather(group).gather(np.asarray(local_rewards, dtype=np.float64).ravel())
    got = np.asarray(gathered, dtype=np.float64).ravel()
    ok = bool(got.shape == want.shape and np.array_equal(got, want))
    return ok, all(group.allgather_bool(ok))


class GlooRewardGather:
    """All-gather of per-env rewards over an initialised torch.distributed group."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self._out = None

    def gather(self, local_rewards):
        import torch
        dist = self.dist
        local = torch.from_numpy(np.ascontiguousarray(local_rewards, dtype=np.float64))
        world = dist.get_world_size(self.group)
        n = torch.tensor([local.numel()], dtype=torch.int64)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, n, group=self.group)
        width = int(max(s.item() for s in sizes))
        padded = torch.zeros(width, dtype=torch.float64)
        padded[:local.numel()] = local
        parts = [torch.zeros(width, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, padded, group=self.group)
        return np.concatenate([p[:int(s.item())].numpy() for p, s in zip(parts, sizes)])
