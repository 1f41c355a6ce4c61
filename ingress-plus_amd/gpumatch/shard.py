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


# ---------------------------------------------------------------- a sharded request stream
# BASELINE.json configs[4] (C5): a 100M-request stream sharded over the GPUs of one node, the
# per-location / per-rule hit counters all-reduced.  Every rank runs the same three pieces: its
# contiguous slice of the stream (shard_bounds), that slice in batches, and the out-of-place
# counter reduction after every step.  bench.py --config c5 drives them with libgpumatch and RCCL;
# tests/test_multi_cpu.py with the CPU oracle and gloo -- the same functions either way.

def stream_records(pool_reqs: np.ndarray, pool_arena_len: int, lo: int, hi: int):
    """The records of stream positions [lo, hi) of a stream that repeats a P-request pool (position
    i = pool record i % P of copy i // P; copy k's arena at k * plen, plen = the pool arena rounded
    up to 16 B).  Returns (reqs, plen, first_copy, n_copies, arena_len): bases are rebased so the
    slice's arena starts at copy first_copy -- lay out copies first_copy .. + n_copies from 0."""
    P = len(pool_reqs)
    plen = (pool_arena_len + 15) & ~15
    if hi <= lo:
        return pool_reqs[:0].copy(), plen, 0, 0, 0
    idx = np.arange(lo, hi, dtype=np.int64)
    copy_ = idx // P
    first = int(copy_[0])
    reqs = pool_reqs[idx % P].copy()
    reqs["base"] += ((copy_ - first) * plen).astype(np.uint64)
    last = reqs[-1]
    arena_len = int(last["base"]) + sum(int(last[f]) for f in ("uri_len", "args_len", "hdr_len", "body_len",
                                                              "host_len", "method_len", "ruri_len", "raddr_len"))
    return reqs, plen, first, int(copy_[-1]) - first + 1, arena_len


def batch_bounds(lo: int, hi: int, batch: int) -> list:
    """[lo, hi) in consecutive batches of at most `batch` requests."""
    return [(b, min(b + batch, hi)) for b in range(lo, hi, max(1, batch))]


class StreamCounters:
    """A rank's cumulative counters and the job-wide totals, reduced OUT OF PLACE (the contract of
    gm_counters_allreduce, include/gpumatch.h): after step k the totals are the sum over ranks of
    every batch so far, however many reductions ran."""

    def __init__(self, n: int, reduce):
        self.local = np.zeros(n, dtype=np.int64)
        self.total = np.zeros(n, dtype=np.int64)
        self._reduce = reduce          # callable: local counters -> their sum over the ranks

    def add(self, c: np.ndarray):
        self.local += c.astype(np.int64)

    def reduce(self) -> np.ndarray:
        self.total = np.asarray(self._reduce(self.local.copy()), dtype=np.int64)
        return self.total


def run_stream(classify, lo: int, hi: int, batch: int, after_step=None, steps: int = 1):
    """One rank's share of the stream, `steps` times: classify(b0, b1) per batch of its slice (the
    caller keeps or accumulates what it returns), then after_step(step) -- the counter reduction."""
    out = []
    for step in range(1, steps + 1):
        out = [classify(b0, b1) for b0, b1 in batch_bounds(lo, hi, batch)]
        if after_step is not None:
            after_step(step)
    return out
