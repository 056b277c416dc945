"""Multi-GPU helpers: launching, env-id sharding and episode-statistics reduction.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, "gloo" on CPU).
The reference's only parallelism is SubprocVecEnv with 8 worker processes
(/root/reference/run.py:114-122); here the envs of a node are sharded over its GPUs.
Envs are independent, so the data path has no collective: rank r owns global env ids
[offset_r, offset_r + n_r).  Philox keys on the global env id, so every env's trajectory
is the same for any world size.  Collectives are used only to reduce per-episode
statistics (a few doubles) and, for the learners, gradients.
"""
import os
import socket
import subprocess
import sys

import torch


def shard(total_envs, rank, world):
    """(env_id_offset, num_envs) of `rank`: contiguous, sizes differ by at most one."""
    base, extra = divmod(int(total_envs), int(world))
    n = base + (1 if rank < extra else 0)
    off = rank * base + min(rank, extra)
    return off, n


def world_info():
    """(rank, world_size, local_rank) from the torchrun environment (1 process: 0, 1, 0)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def forced_multi():
    """LBK8S_FORCE_MULTI=1: the multi-rank code path (collectives, split graphs) even in a
    one-rank process group -- the RCCL path exercised on a one-GPU box."""
    return os.environ.get("LBK8S_FORCE_MULTI") == "1"


def is_multi():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or forced_multi())


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(nproc, target, argv, module=False):
    """Run `target argv` (a script path, or a module name with module=True) as `nproc`
    ranks of one node (torch.distributed.run, rendezvous on 127.0.0.1) in a CHILD process
    and return its exit code.  The caller must not have touched the GPU: it only spawns and
    waits (no exec from a process that initialised HIP)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(nproc)}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port())]
    cmd += (["-m", target] if module else [target]) + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    pkg_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    return subprocess.run(cmd, env=env).returncode


def init_from_env(device_type="cuda", backend=None):
    """Initialise the default process group from the torchrun environment (no-op for one
    process).  GPUs: one per rank (LOCAL_RANK), backend nccl (= RCCL); CPU: gloo.
    LBK8S_DIST_BACKEND=gloo overrides the backend: with it, ranks beyond the visible GPUs
    share them (LOCAL_RANK mod device count) — a test mode for a one-GPU box.  With
    LBK8S_FORCE_MULTI=1 a single process forms a one-rank group (RCCL on a GPU).
    Returns (rank, world, device)."""
    import torch.distributed as dist
    rank, world, local = world_info()
    backend = backend or os.environ.get("LBK8S_DIST_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    if device_type == "cuda":
        idx = local % max(torch.cuda.device_count(), 1) if backend == "gloo" else local
        dev = torch.device("cuda", idx)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if (world > 1 or forced_multi()) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:  # (a one-rank group outside torchrun)
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return rank, world, dev


def all_reduce_sum(t, group=None):
    """In-place SUM over ranks (no-op for one process); returns t."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def reduce_episode_stats(ep_stats, dones, group=None):
    """Sum, over all ranks, of (episodes finished, return, length, accepted) for the envs
    that finished this step.  ep_stats (B, 16) float64, dones (B,) bool/uint8 (any device).
    Returns a float64 tensor [count, sum_return, sum_length, sum_accepted] on the same device.
    """
    d = dones.to(torch.bool)
    rows = ep_stats[d]
    v = torch.stack([d.sum().to(torch.float64), rows[:, 0].sum(), rows[:, 1].sum(), rows[:, 2].sum()])
    return all_reduce_sum(v, group)


def mean_episode_return(ep_sum, ep_cnt, group=None):
    """Global mean finished-episode return from per-rank (sum, count) device accumulators
    (any shape; summed) — the learners' logged ep_return.  One 2-double all_reduce."""
    v = torch.stack([ep_sum.sum().to(torch.float64), ep_cnt.sum().to(torch.float64)])
    all_reduce_sum(v, group)
    s, n = v.tolist()
    return (s / n if n > 0 else None), n


def broadcast_parameters(module, src=0, group=None):
    """Copy rank src's parameters to every rank (one flat broadcast)."""
    import torch.distributed as dist
    if not is_multi():
        return
    params = list(module.parameters())
    flat = torch.cat([p.detach().reshape(-1) for p in params])
    dist.broadcast(flat, src=src, group=group)
    off = 0
    with torch.no_grad():
        for p in params:
            n = p.numel()
            p.copy_(flat[off:off + n].view_as(p))
            off += n
