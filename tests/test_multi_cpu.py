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


# ---------------------------------------------------------------- C5: a sharded request stream
# BASELINE.json configs[4] through the same gpumatch.shard code bench.py --config c5 runs with
# libgpumatch and RCCL: stream_records (a rank's contiguous slice of a stream that repeats a
# pool), run_stream (the slice in batches, a counter reduction after every step) and
# StreamCounters (cumulative local counters, out-of-place totals).  The oracle classifies and
# gloo reduces here.
C5_STREAM, C5_POOL, C5_BATCH = 5000, 1700, 700


def _c5_pool():
    return workloads.c5_blob(n_hosts=60), workloads.gen_c5(C5_POOL, n_hosts=60)


def _c5_arena(parena, plen, ncopies):
    a = np.zeros(ncopies * plen, dtype=np.uint8)
    for k in range(ncopies):
        a[k * plen:k * plen + len(parena)] = parena
    return a


def _c5_rank(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blob, (preqs, parena) = _c5_pool()
    o = Oracle(blob, 1)
    n_locs = 4096   # >= the generation's locations (60 hosts x <= 8 minions x <= 2 paths)
    lo, hi = shard.shard_bounds(C5_STREAM, world, rank)
    reqs, plen, first, ncopies, alen = shard.stream_records(preqs, len(parena), lo, hi)
    arena = _c5_arena(parena, plen, ncopies)

    def reduce(x):
        t = torch.from_numpy(x)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.numpy()
    ctr = shard.StreamCounters(n_locs, reduce)
    verdicts = {}

    def classify(b0, b1):
        v, _ = o.match(reqs[b0:b1], arena, nthreads=1)
        loc = v["location_id"][v["location_id"] != 0xFFFFFFFF].astype(np.int64)
        ctr.add(np.bincount(loc, minlength=n_locs))
        verdicts[b0] = v
        return v

    def after_step(step):
        tot = ctr.reduce()
        if rank == 0:
            np.save(os.path.join(out_dir, f"c5_counters_{step}.npy"), tot)
    shard.run_stream(classify, 0, hi - lo, C5_BATCH, after_step, steps=2)
    mine = np.concatenate([verdicts[k] for k in sorted(verdicts)])
    gathered = [None] * world
    dist.all_gather_object(gathered, mine.tobytes())
    if rank == 0:
        np.save(os.path.join(out_dir, "c5_verdicts.npy"),
                np.concatenate([np.frombuffer(b, dtype=records.VERDICT_DTYPE) for b in gathered]))
    dist.destroy_process_group()


def test_stream_records_slices_the_repeated_pool():
    """Stream positions map to (copy, pool record): a slice's records are the pool's, rebased onto
    the copies the slice spans."""
    _, (preqs, parena) = _c5_pool()
    full, plen, f0, n0, alen0 = shard.stream_records(preqs, len(parena), 0, C5_STREAM)
    assert f0 == 0 and n0 == (C5_STREAM + C5_POOL - 1) // C5_POOL
    for lo, hi in [(0, 10), (1690, 1720), (3400, 5000), (777, 777)]:
        part, _, first, ncopies, alen = shard.stream_records(preqs, len(parena), lo, hi)
        if hi == lo:
            assert len(part) == 0 and ncopies == 0
            continue
        assert np.array_equal(part["uri_len"], full["uri_len"][lo:hi])
        assert np.array_equal(part["base"] + np.uint64(first * plen), full["base"][lo:hi])
        assert first == lo // C5_POOL and first + ncopies - 1 == (hi - 1) // C5_POOL


def test_two_rank_gloo_c5_stream_matches_single_process(tmp_path):
    mp.spawn(_c5_rank, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    blob, (preqs, parena) = _c5_pool()
    reqs, plen, _, ncopies, _ = shard.stream_records(preqs, len(parena), 0, C5_STREAM)
    v, _ = Oracle(blob, 1).match(reqs, _c5_arena(parena, plen, ncopies), nthreads=2)
    got = np.load(tmp_path / "c5_verdicts.npy")
    assert got.tobytes() == v.tobytes()
    loc = v["location_id"][v["location_id"] != 0xFFFFFFFF].astype(np.int64)
    one = np.bincount(loc, minlength=4096)
    for step in (1, 2):
        assert np.array_equal(np.load(tmp_path / f"c5_counters_{step}.npy"), step * one)
    assert one.sum() > C5_STREAM // 10   # about half the stream is plain http: redirected before a location


# ---------------------------------------------------------------- generation agreement
# gm_counters_allreduce carries the ranks' agreement on (gen, n_counters) inside the counter SUM
# itself: a block {1, v, v^2 over the 16-bit halves of gen and n} beside the counters, one
# collective of RED_WORDS + the agreed count on every rank and no host round trip (VERDICT r5 item
# 4).  A call whose block shows the ranks apart has no totals (GM_E_COMM on every rank) and the next
# call re-agrees synchronously (a block-only collective) before any sum.  These tests drive the
# library's own state machine (gm_debug_red_*) with gloo as the transport, RCCL on the GPU: every
# rank takes the same branch at every call, and no collective of mismatched size is ever issued (a
# size mismatch would fail the gloo all_reduce here).
def _agree_rank(rank, world, port, out_dir, gens):
    import ctypes
    from gpumatch import engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L = engine.lib()
    L.gm_debug_red_words.restype = ctypes.c_uint32
    L.gm_debug_red_pack.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    L.gm_debug_red_new.restype = ctypes.c_void_p
    L.gm_debug_red_free.argtypes = [ctypes.c_void_p]
    L.gm_debug_red_begin.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    L.gm_debug_red_agree.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    L.gm_debug_red_finish.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    W = L.gm_debug_red_words()
    proto = L.gm_debug_red_new()

    def words(t):
        return (ctypes.c_uint64 * W)(*[int(x) for x in t[:W].tolist()])
    results = []
    for gen, blob in gens[rank]:
        e = engine.Engine(compile_only=True)
        e.load(blob, gen)
        st = e.stats()
        blk = (ctypes.c_uint64 * W)()
        L.gm_debug_red_pack(st["gen"], st["n_counters"], blk)
        count = ctypes.c_uint64(0)
        agreed_now = False
        if L.gm_debug_red_begin(proto, ctypes.byref(count)):   # synchronous agreement first
            t = torch.tensor(list(blk), dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            rc = L.gm_debug_red_agree(proto, words(t))
            if rc != 0:
                results.append((rc, -1, 1))
                e.close()
                continue
            agreed_now = True
            L.gm_debug_red_begin(proto, ctypes.byref(count))
        # the combined collective: the block + this rank's counters (ones) cut / padded to the count
        n = int(count.value)
        c = torch.zeros(W + n, dtype=torch.int64)
        c[:W] = torch.tensor(list(blk), dtype=torch.int64)
        c[W:W + min(n, st["n_counters"])] = 1
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        rc = L.gm_debug_red_finish(proto, words(c))
        results.append((rc, int(c[W]) if rc == 0 else -1, int(agreed_now)))
        e.close()
    L.gm_debug_red_free(proto)
    np.save(os.path.join(out_dir, f"agree_{rank}.npy"), np.array(results, dtype=np.int64))
    dist.destroy_process_group()


def test_two_rank_generation_agreement(tmp_path):
    """Ranks on different generations (call 1) or counter spaces (call 2): GM_E_COMM on both ranks
    at the same call, the re-agreement at the next call, then totals again (call 3)."""
    from gpumatch import engine
    a = workloads.c4_blob(workloads.c4_sigset(400, 100), "monitoring")
    b = workloads.c4_blob(workloads.c4_sigset(300, 50), "monitoring")   # another counter space
    gens = {0: [(1, a), (2, a), (3, a), (4, a)],
            1: [(1, a), (3, a), (3, b), (4, a)]}
    mp.spawn(_agree_rank, args=(2, _free_port(), str(tmp_path), gens), nprocs=2, join=True)
    r0, r1 = np.load(tmp_path / "agree_0.npy"), np.load(tmp_path / "agree_1.npy")
    assert np.array_equal(r0, r1)   # every rank takes the same branch
    assert r0[:, 0].tolist() == [0, engine.GM_E_COMM, engine.GM_E_COMM, 0]
    assert r0[0, 1] == 2 and r0[3, 1] == 2
    # only the first call and the calls after a failure agree synchronously (a host round trip)
    assert r0[:, 2].tolist() == [1, 0, 1, 1]


def test_two_rank_steady_state_is_one_collective(tmp_path):
    """Steady state: after the first call's agreement every call is one combined collective with no
    synchronous agreement; a reload every rank makes together keeps the totals valid (same counter
    space), a new counter space on every rank costs one call's totals and one re-agreement."""
    from gpumatch import engine
    a = workloads.c4_blob(workloads.c4_sigset(400, 100), "monitoring")
    b = workloads.c4_blob(workloads.c4_sigset(300, 50), "monitoring")
    seq = [(1, a), (1, a), (2, a), (3, b), (4, b), (4, b)]
    mp.spawn(_agree_rank, args=(2, _free_port(), str(tmp_path), {0: seq, 1: seq}), nprocs=2, join=True)
    r0, r1 = np.load(tmp_path / "agree_0.npy"), np.load(tmp_path / "agree_1.npy")
    assert np.array_equal(r0, r1)
    assert r0[:, 0].tolist() == [0, 0, 0, engine.GM_E_COMM, 0, 0]
    assert r0[:, 2].tolist() == [1, 0, 0, 0, 1, 0]
    assert (r0[r0[:, 0] == 0, 1] == 2).all()
