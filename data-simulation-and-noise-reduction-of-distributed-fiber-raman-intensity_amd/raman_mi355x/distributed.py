"""Data-parallel helpers: one process per GPU, spectra sharded by contiguous index range.

Spectra are independent and weights are replicated, so there is no exchange during compute
(SURVEY.md §8e).  The only collective of an evaluation is the all-reduce of the fp64 metric sums
{ΣMSE, ΣSSIM, ΣSmoothness, ΣPeak2Peak, count} — RCCL ("nccl" backend) over xGMI on MI355X,
gloo for CPU tensors.  Because the simulator is counter-based (spectrum i is the same on every
device), the sharded data set is identical for any world size.
"""
import torch
import torch.distributed as dist


def world():
    """(rank, world_size) of the default process group, (0, 1) when not distributed."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard(n, rank=None, world_size=None):
    """Contiguous [start, stop) of n items owned by `rank` (balanced to within one item)."""
    if rank is None or world_size is None:
        rank, world_size = world()
    if not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} outside world of size {world_size}")
    return n * rank // world_size, n * (rank + 1) // world_size


def all_reduce_sums(sums):
    """In-place SUM all-reduce of a metric-sum tensor (no-op when not distributed)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
    return sums


def means(sums):
    """{MSE, SSIM, Smoothness, Peak2Peak} means from the 5-vector of sums (evaulate.py:39)."""
    s = [float(v) for v in sums.tolist()]
    if s[4] <= 0:
        raise ValueError("no spectra were evaluated")
    return {k: s[i] / s[4] for i, k in enumerate(("MSE", "SSIM", "Smoothness", "Peak2Peak"))}
