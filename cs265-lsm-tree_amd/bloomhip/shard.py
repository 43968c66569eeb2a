"""Per-run sharding across GPUs.

Filters of different LSM runs are independent (one per run, src/run.h:10-30),
so builds shard one run per GPU with no exchange step: run r is built on rank
r mod world.  Probes replicate the filters on every GPU and shard the GET
keys contiguously (probe_slice): the ranks' result slices are disjoint.  The only collectives are bookkeeping: the max over ranks of a
timed region and an all-gather of per-run digests for verification.  They use
whatever torch.distributed backend the caller initialised (RCCL on GPUs,
gloo on CPU).
"""
from __future__ import annotations

import hashlib
from typing import Callable, Dict, Iterable, List, Tuple


def rank_for_run(run: int, world: int) -> int:
    return run % world


def runs_for_rank(n_runs: int, rank: int, world: int) -> List[int]:
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world {world}")
    return [r for r in range(n_runs) if rank_for_run(r, world) == rank]


def digest(words) -> str:
    import numpy as np
    return hashlib.sha256(np.ascontiguousarray(words).tobytes()).hexdigest()


def build_my_runs(n_runs: int, rank: int, world: int,
                  build: Callable[[int], "object"]) -> Dict[int, str]:
    """Build this rank's runs with `build(run) -> bitmap words`; digests by run."""
    return {r: digest(build(r)) for r in runs_for_rank(n_runs, rank, world)}


def gather_digests(local: Dict[int, str], dist) -> Dict[int, str]:
    """All-gather every rank's {run: digest}; returns the union (same on every rank)."""
    world = dist.get_world_size()
    parts: List[Dict[int, str]] = [None] * world  # type: ignore[list-item]
    dist.all_gather_object(parts, local)
    out: Dict[int, str] = {}
    for p in parts:
        for r, d in p.items():
            if r in out:
                raise RuntimeError(f"run {r} built on two ranks")
            out[r] = d
    return out


def max_over_ranks(value: float, dist, device=None) -> float:
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: int, dist, device=None) -> int:
    import torch
    t = torch.tensor([value], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def all_ranks_ok(ok: bool, dist, device=None) -> bool:
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def probe_slice(n_keys: int, rank: int, world: int, align: int = 64) -> Tuple[int, int]:
    """The contiguous slice of a GET burst that `rank` probes (SURVEY §8e:
    filters replicated on every GPU, keys sharded).  Slice bounds are
    multiples of `align` (64: one packed result word never straddles two
    ranks), so the ranks' packed result rows concatenate into the whole."""
    if world <= 0 or not 0 <= rank < world or align <= 0:
        raise ValueError(f"bad rank {rank} for world {world}")
    units = (n_keys + align - 1) // align
    lo_u, hi_u = units * rank // world, units * (rank + 1) // world
    return min(n_keys, lo_u * align), min(n_keys, hi_u * align)


def covers(runs: Iterable[int], n_runs: int) -> bool:
    return sorted(runs) == list(range(n_runs))
