"""Multi-GPU helpers for bench.py (weak scaling, no data-path collective: SURVEY.md 8(e)).

Rank r of W owns the contiguous tuple range [r*N, (r+1)*N) of the synthetic workload; the
only cross-rank traffic is the barrier around the timed region and one MAX reduction of the
elapsed time (plus a SUM of parity mismatches)."""
from __future__ import annotations


def shard_range(rank: int, world: int, per_rank: int) -> tuple[int, int]:
    assert 0 <= rank < world and per_rank >= 0
    return rank * per_rank, (rank + 1) * per_rank


def reduce_timing(elapsed: float, mismatches: int, device=None) -> tuple[float, int]:
    """MAX of elapsed seconds and SUM of mismatches over all ranks (no-op when not distributed)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return elapsed, mismatches
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    m = torch.tensor([mismatches], dtype=torch.int64, device=device)
    dist.all_reduce(m)
    return float(t.item()), int(m.item())
