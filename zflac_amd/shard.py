"""Stream sharding across ranks (one process per GPU) and the job-level aggregation.

FLAC streams are independent objects, so the multi-GPU path is pure sharding: rank r
decodes streams [r * n, (r + 1) * n) of the job with no data-path collective. The only
collectives are the timing barrier, the max of the per-rank elapsed time and the sums of
the per-rank counters (torch.distributed; "nccl" is RCCL on ROCm, "gloo" on CPU).
"""
from __future__ import annotations

from dataclasses import dataclass


def shard_range(rank: int, world: int, per_rank: int) -> range:
    """Global stream indices owned by `rank` (weak scaling: fixed work per rank)."""
    if not (0 <= rank < world) or per_rank < 0:
        raise ValueError(f"bad shard request rank={rank} world={world} per_rank={per_rank}")
    return range(rank * per_rank, (rank + 1) * per_rank)


@dataclass
class JobTotals:
    elapsed_s: float   # max over ranks
    samples: float     # sum over ranks (per step)
    input_bytes: float
    output_bytes: float
    errors: int        # sum over ranks


def aggregate(dist, device, elapsed_s: float, samples: int, input_bytes: int, output_bytes: int,
              errors: int) -> JobTotals:
    """Job totals over all ranks; `dist` is torch.distributed (initialised) or None."""
    if dist is None:
        return JobTotals(elapsed_s, float(samples), float(input_bytes), float(output_bytes), int(errors))
    import torch

    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([float(samples), float(input_bytes), float(output_bytes), float(errors)],
                     dtype=torch.float64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    v = s.tolist()
    return JobTotals(float(t.item()), v[0], v[1], v[2], int(round(v[3])))
