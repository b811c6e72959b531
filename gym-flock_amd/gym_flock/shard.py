"""Multi-GPU sharding of the env batch.

Envs are independent, so the batch is split into contiguous ranges, one per rank
(one process per GPU); the step path has no exchange. The only collective is the
metrics path: per-env rewards are all-gathered so every rank (or the trainer on
rank 0) sees the whole batch's rewards in global env order; optionally the per-env
get_stats summaries (means of vel_diffs and min_dists) likewise.

Transports for that all-gather:
  - RcclRewardGather: RCCL over xGMI, issued by libgymflock on a side stream right
    after the step kernel (fe_allgather_rewards) — the GPU path. Each rank's block is
    padded to the largest shard (pad_block's layout); unpad_gathered restores the global
    env order, so shard_range's uneven splits work unchanged.
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


def pad_block(local, width, axis=0):
    """A rank's per-env array padded with zeros to `width` envs along `axis`: the block
    layout of the RCCL gathers (include/gymflock.h: every rank ships max_envs columns,
    those past its own n_envs zero)."""
    local = np.asarray(local, dtype=np.float64)
    pad = [(0, 0)] * local.ndim
    pad[axis] = (0, int(width) - local.shape[axis])
    return np.pad(local, pad)


def unpad_gathered(blocks, sizes, axis=0):
    """Rank-major gathered blocks, each padded to the largest shard, -> global env order:
    rank r's first sizes[r] entries along `axis` (the env axis of one rank's block),
    concatenated in rank order."""
    blocks = np.asarray(blocks)
    if len(blocks) != len(sizes):
        raise ValueError("%d gathered blocks for %d ranks" % (len(blocks), len(sizes)))
    return np.concatenate([np.take(b, np.arange(n), axis=axis) for b, n in zip(blocks, sizes)], axis=axis)


class RcclRewardGather:
    """All-gather of per-env rewards with RCCL; shards may differ in size (the library
    pads every rank's block to the largest shard, result() drops the padding).

    issue() after a step enqueues one collective carrying every step since the previous
    issue() (at any interval up to 64 steps); result() returns them as (steps, total_envs)
    in global env order."""

    def __init__(self, handle, world_size, rank, unique_id, timeout=300.0):
        self.handle = handle
        handle.comm_init(world_size, rank, unique_id, timeout)
        self.sizes = handle.shard_sizes

    def issue(self):
        self.handle.allgather_rewards()

    def result(self):
        return unpad_gathered(self.handle.gathered_rewards(), self.sizes, axis=1)  # (world, steps, W)

    def issue_stats(self):
        """The optional get_stats aggregates: every rank's per-env means of
        vel_diffs and min_dists of the current state, all-gathered on the side stream."""
        self.handle.allgather_stats()

    def stats_result(self):
        """(total_envs, 2) per-env [mean vel_diffs, mean min_dists] in global env order."""
        return unpad_gathered(self.handle.gathered_stats(), self.sizes, axis=0)  # (world, W, 2)

    def comm_info(self):
        """The communicator as RCCL reports it on this rank (fe_comm_info)."""
        return self.handle.comm_info()


def exchange_shard_sizes(group, n_envs):
    """Every rank's env count over the host channel (in rank order, on every rank)."""
    sizes = group.allgather_i64(int(n_envs))
    if min(sizes) < 1:
        raise RuntimeError("bad env shard sizes over ranks: n_envs per rank = %s" % sizes)
    return sizes


def init_rccl_gather(group, handle, world, rank, timeout=300.0):
    """The multi-rank path's RCCL setup, bounded by the host channel: the ranks' shard
    sizes are exchanged first; rank 0's unique id goes out only once every rank has joined
    the channel (HostGroup's rendezvous); each rank's bounded communicator init
    (fe_comm_init_timeout) reports success over the channel, and every rank raises if any
    rank failed, instead of leaving the others in RCCL. Returns an RcclRewardGather."""
    sizes = exchange_shard_sizes(group, handle.n_envs)
    uid = group.broadcast_bytes(handle.comm_unique_id() if rank == 0 else b"")
    err = None
    try:
        gather = RcclRewardGather(handle, world, rank, uid, timeout)
        if gather.sizes != sizes:
            raise RuntimeError("RCCL's shard-size exchange %s differs from the host channel's %s"
                               % (gather.sizes, sizes))
    except Exception as e:  # reported to every rank below, then re-raised here
        err, gather = e, None
    ok = group.allgather_bool(err is None)
    if err is not None:
        raise err
    if not all(ok):
        raise RuntimeError("RCCL communicator init failed on rank(s) %s" % [r for r, v in enumerate(ok) if not v])
    return gather


def rccl_report(group, gather, world):
    """Every rank's communicator as RCCL reports it, collected on every rank, with the
    checks rank 0 makes before it reports a multi-rank figure: ncclCommCount equals the
    number of ranks everywhere, the user ranks are 0..world-1 in order, and no two ranks
    share a device PCI bus id (one process per GPU). Raises if any check fails."""
    import json
    mine = json.dumps(gather.comm_info(), sort_keys=True).encode()
    infos = [json.loads(p.decode()) for p in group.allgather_bytes(mine)]
    problems = []
    if any(i["count"] != world for i in infos):
        problems.append("ncclCommCount %s != %d ranks" % ([i["count"] for i in infos], world))
    if [i["user_rank"] for i in infos] != list(range(world)):
        problems.append("user ranks %s" % [i["user_rank"] for i in infos])
    buses = [i["pci_bus_id"] for i in infos]
    if len(set(buses)) != len(buses):
        problems.append("ranks share a GPU: PCI bus ids %s" % buses)
    if problems:
        raise RuntimeError("RCCL communicator check failed: " + "; ".join(problems))
    return {"ranks": infos, "count": world, "distinct_devices": len(set(buses)),
            "shard_sizes": list(gather.sizes)}


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
