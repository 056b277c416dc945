"""Multi-GPU helpers: env-id sharding and episode-statistics reduction.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, "gloo" on CPU).
Envs are independent, so the data path has no collective: rank r owns global env ids
[offset_r, offset_r + n_r).  Philox keys on the global env id, so every env's trajectory
is the same for any world size.  Collectives are used only to reduce per-episode
statistics (a few doubles) and, for the learners, gradients.
"""
import torch


def shard(total_envs, rank, world):
    """(env_id_offset, num_envs) of `rank`: contiguous, sizes differ by at most one."""
    base, extra = divmod(int(total_envs), int(world))
    n = base + (1 if rank < extra else 0)
    off = rank * base + min(rank, extra)
    return off, n


def reduce_episode_stats(ep_stats, dones, group=None):
    """Sum, over all ranks, of (episodes finished, return, length, accepted) for the envs
    that finished this step.  ep_stats (B, 16) float64, dones (B,) bool/uint8 (any device).
    Returns a float64 tensor [count, sum_return, sum_length, sum_accepted] on the same device.
    """
    import torch.distributed as dist
    d = dones.to(torch.bool)
    rows = ep_stats[d]
    v = torch.stack([d.sum().to(torch.float64), rows[:, 0].sum(), rows[:, 1].sum(), rows[:, 2].sum()])
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(v, op=dist.ReduceOp.SUM, group=group)
    return v
