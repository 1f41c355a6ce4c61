"""Request sharding for one process per GPU (SURVEY.md §8 e).

Requests are independent: a stream of N records splits into contiguous chunks, one per rank, so
verdicts keep their global order when the per-rank outputs are concatenated.  The rule set is
replicated (every rank loads the same generation) and the only cross-rank step is the sum of
the per-location / per-rule hit counters (gm_counters_allreduce, RCCL over xGMI on the GPUs).
"""

from __future__ import annotations

import numpy as np


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of request indices owned by `rank` (sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return n * rank // world, n * (rank + 1) // world


def slice_batch(reqs: np.ndarray, arena: np.ndarray, lo: int, hi: int):
    """Records [lo, hi) with their own arena (bases rebased, 16-B alignment kept)."""
    part = reqs[lo:hi].copy()
    if len(part) == 0:
        return part, np.zeros(0, dtype=np.uint8)
    start = int(part["base"][0])
    end = int(reqs["base"][hi]) if hi < len(reqs) else len(arena)
    part["base"] -= np.uint64(start)
    return part, np.ascontiguousarray(arena[start:end])


def merge_hits(verdicts: list[np.ndarray], hits: list[np.ndarray]):
    """Concatenate per-shard verdicts and hit-id lists into the single-batch layout
    (first_hit_off re-based onto the concatenated hit list)."""
    out, off = [], 0
    for v, h in zip(verdicts, hits):
        v = v.copy()
        v["first_hit_off"] = np.where(v["n_hits"] > 0, v["first_hit_off"] + off, v["first_hit_off"])
        out.append(v)
        off += len(h)
    return (np.concatenate(out) if out else np.zeros(0)), (np.concatenate(hits) if hits else np.zeros(0))
