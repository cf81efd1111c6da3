"""Object -> GPU partitioning for the multi-GPU path.

Storb's erasure stage is embarrassingly parallel: every object (and every
chunk of an object) encodes and decodes independently, so N GPUs of one
node split the objects round-robin -- object i goes to rank i mod N -- and
never exchange data (no RCCL collective on the data path). The only
cross-rank traffic is the benchmark's barrier and max-over-ranks timing.
"""
from __future__ import annotations

from typing import Sequence


def owner(obj: int, world: int) -> int:
    """Rank (= GPU) that encodes/decodes object `obj`."""
    return obj % world


def objects_for_rank(nobj: int, rank: int, world: int) -> range:
    """The objects rank `rank` owns: i = rank, rank + world, ..."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return range(rank, nobj, world)


def chunks_of(total: int, chunk: int) -> list[tuple[int, int]]:
    """(offset, length) of each chunk of a `total`-byte object cut at
    `chunk` bytes (upload.rs:333-383); the last chunk may be short."""
    return [(o, min(chunk, total - o)) for o in range(0, total, chunk)]


def aggregate_rate(units_per_rank: Sequence[int], elapsed_per_rank: Sequence[float]) -> float:
    """Whole-job throughput: every rank's units over the slowest rank's time."""
    return float(sum(units_per_rank)) / max(elapsed_per_rank)
