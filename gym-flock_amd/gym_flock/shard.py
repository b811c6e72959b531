"""Multi-GPU sharding of the env batch.

Envs are independent, so the batch is split into contiguous ranges, one per rank
(one process per GPU); the step path has no exchange. The only collective is the
metrics path: per-env rewards are all-gathered so every rank (or the trainer on
rank 0) sees the whole batch's rewards in global env order.

Two transports for that all-gather:
  - RcclRewardGather: RCCL over xGMI, issued by libgymflock on a side stream right
    after the step kernel (fe_allgather_rewards) — the GPU path.
  - GlooRewardGather: torch.distributed (gloo) on host copies — used by the CPU
    tests and by callers that already hold a gloo group.
torch is imported lazily and only by the gloo transport: the env itself has no
PyTorch dependency.
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

    def __init__(self, handle, world_size, rank, unique_id):
        self.handle = handle
        handle.comm_init(world_size, rank, unique_id)

    def issue(self):
        self.handle.allgather_rewards()

    def result(self):
        g = self.handle.gathered_rewards()  # (world, steps, B)
        return np.concatenate(list(g), axis=1)


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
