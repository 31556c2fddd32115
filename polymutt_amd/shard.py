"""Site sharding across GPUs.

Sites are independent, so each rank (one process per GPU) takes a contiguous range of sites of a
section and runs the engine on it; nothing crosses ranks on the data path.  The only cross-site
state is the section summary counters (src/main.cpp:264-282), combined with ONE all-reduce(sum) of
the 16 int64 pm_counters fields at the end of a section -- RCCL over xGMI on GPUs (backend "nccl"),
gloo in the CPU tests.
"""
import numpy as np


def shard_range(n_sites, rank, world):
    """Contiguous [lo, hi) slice of n_sites for `rank` (keeps VCF order when shards are concatenated)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(n_sites, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def allreduce_counters(counters, device=None):
    """Sum a section's counters (pm_counters as int64[16]) over all ranks of the default process group.

    `device` is where the reduction buffer lives: a CUDA device for RCCL, None (CPU) for gloo."""
    import torch
    import torch.distributed as dist
    t = torch.as_tensor(np.asarray(counters, dtype=np.int64).copy(), device=device)
    if dist.is_available() and dist.is_initialized():   # (also at one rank: an RCCL group of one still runs it)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (timing: the job is as slow as its slowest rank)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
