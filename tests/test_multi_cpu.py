"""N > 1 path on the CPU: world_size-2 `gloo` ranks shard a C4 batch with gpumatch.shard,
classify their shard (the oracle stands in for the GPU here), all-reduce the per-location and
per-rule counters, and gather the verdicts.  The merged result must equal the single-process
batch bit for bit, and the reduced counters must equal its counters (SURVEY.md §8 e).

Counters follow libgpumatch's contract (include/gpumatch.h gm_counters_allreduce): each rank's
counters are cumulative over its batches, and every reduction is OUT OF PLACE into a separate
buffer -- so after step k the reduced totals are exactly k x the single-process counters (an
in-place reduction of cumulative counters would double-count from the second call on)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gpumatch import records, shard, workloads
from oracle_py import Oracle

N = 3000
STEPS = 2


def _batch():
    ss = workloads.c4_sigset(400, 100)
    reqs, arena = records.gen_c4(N, ss, plant_rate=0.1)
    return workloads.c4_blob(ss, "monitoring"), reqs, arena, len(ss.rules)


def _counters(verdicts, hits, n_locs, n_rules):
    loc = verdicts["location_id"][verdicts["location_id"] != 0xFFFFFFFF].astype(np.int64)
    return np.concatenate([np.bincount(loc, minlength=n_locs),
                           np.bincount(hits.astype(np.int64), minlength=n_rules)]).astype(np.int64)


def _rank(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blob, reqs, arena, n_rules = _batch()
    lo, hi = shard.shard_bounds(len(reqs), world, rank)
    part, parena = shard.slice_batch(reqs, arena, lo, hi)
    local = torch.zeros(8 + n_rules, dtype=torch.int64)   # this rank's cumulative counters
    for step in range(1, STEPS + 1):
        v, h = Oracle(blob, 1).match(part, parena, nthreads=2)
        local += torch.from_numpy(_counters(v, h, 8, n_rules))
        c = local.clone()                                    # out of place: `local` stays this rank's
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        if rank == 0:
            np.save(os.path.join(out_dir, f"counters_{step}.npy"), c.numpy())
    gathered = [None] * world
    dist.all_gather_object(gathered, (v.tobytes(), h.tobytes()))
    if rank == 0:
        vs = [np.frombuffer(b, dtype=records.VERDICT_DTYPE) for b, _ in gathered]
        hs = [np.frombuffer(x, dtype=np.uint32) for _, x in gathered]
        mv, mh = shard.merge_hits(vs, hs)
        np.save(os.path.join(out_dir, "verdicts.npy"), mv)
        np.save(os.path.join(out_dir, "hits.npy"), mh)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_and_balance():
    for n in (0, 1, 7, 1000):
        for world in (1, 2, 3, 8):
            b = [shard.shard_bounds(n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1


def test_two_rank_gloo_shards_match_single_batch(tmp_path):
    mp.spawn(_rank, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    blob, reqs, arena, n_rules = _batch()
    v, h = Oracle(blob, 1).match(reqs, arena, nthreads=2)
    mv = np.load(tmp_path / "verdicts.npy")
    mh = np.load(tmp_path / "hits.npy")
    assert mv.tobytes() == v.tobytes()
    assert np.array_equal(mh, h)
    for step in range(1, STEPS + 1):
        assert np.array_equal(np.load(tmp_path / f"counters_{step}.npy"), step * _counters(v, h, 8, n_rules))
    assert len(h) > 0
