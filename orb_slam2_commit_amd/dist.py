"""Multi-GPU plumbing for the frame-sharded hot path.

Extraction + stereo matching of a frame is a pure function of that frame, so
frames shard across ranks with no data-path collective; the only
communication is the benchmark's barrier and the max-over-ranks of the timed
region (torch.distributed; backend "nccl" = RCCL on ROCm, "gloo" in CPU tests).
"""
import os


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend, rank, world):
    import torch.distributed as dist
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        dist.init_process_group(backend, rank=rank, world_size=world)
    return world > 1


def frame_seeds(rank, n_unique):
    """Distinct synthetic stereo scenes per rank (each rank owns its frame shard)."""
    return [1000 * rank + s for s in range(n_unique)]


def _coll_device(device):
    """Collective tensors live on the GPU for RCCL, on the CPU for gloo."""
    import torch.distributed as dist
    return None if dist.get_backend() == "gloo" else device


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (the slowest rank defines the job time)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    device = _coll_device(device)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, device=None):
    """Sum of a float over all ranks (work done by the whole job)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    device = _coll_device(device)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def distinct_devices(local_index, device=None):
    """Number of distinct GPUs the ranks of this (one-node) job run on: every rank contributes its
    device index, rank 0 counts the distinct values.  One rank: 1."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return 1
    device = _coll_device(device)
    t = torch.tensor([int(local_index)], dtype=torch.int64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return len({int(x.item()) for x in out})


def backend():
    """The initialised process group's backend ("nccl" = RCCL, "gloo"), None for one rank."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_backend()
    return None


def barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def job_throughput(frames_per_rank_per_step, steps, world, elapsed_max):
    """Whole-job frames/s: every rank's frames over the slowest rank's time."""
    return frames_per_rank_per_step * steps * world / elapsed_max
