"""The boundary's pipeline properties on the GPU, through libgpumatch.so:

- the benchmarked workload itself (bench.py's C4 generation and its 1M-request pool, replicated
  x10 in HBM) against the oracle, and every HBM replica identical;
- gm_match_batch is asynchronous (returns before the device finishes) and thread-safe per
  (ctx, stream): two batches on two streams, each checked against the oracle;
- counters: cumulative per device, the RCCL reduction out of place (N calls = true totals);
- status hygiene: a normalisation after an overflowing batch syncs clean.
"""

import threading

import numpy as np
import pytest

from gpumatch import engine, records, workloads
from helpers import assert_verdicts_equal
from oracle_py import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    return torch, torch.device("cuda", 0)


def _to_dev(torch, dev, reqs, arena, extra=1024):
    d_reqs = torch.from_numpy(np.ascontiguousarray(reqs).view(np.uint8).reshape(-1)).to(dev)
    d_arena = torch.zeros(len(arena) + extra, dtype=torch.uint8, device=dev)
    if len(arena):
        d_arena[:len(arena)].copy_(torch.from_numpy(np.ascontiguousarray(arena)))
    return d_reqs, d_arena


def _split_hits(v, hits):
    return [hits[int(o):int(o) + int(k)] for o, k in zip(v["first_hit_off"], v["n_hits"])]


def test_benched_c4_pool_parity_and_replicas(torch_dev):
    """bench.py's exact workload: 200k requests of the 1M-request pool against the oracle, and all
    ten HBM replicas of the pool (10M requests, one batch) give identical verdicts and hit lists."""
    torch, dev = torch_dev
    ss, gblob = workloads.c4_bench_generation()
    preqs, parena = records.gen_c4(1_000_000, ss, seed=workloads.C4_POOL_SEED)
    n = 10_000_000
    reqs, plen, reps, arena_len = workloads.replicate_pool(preqs, len(parena), n)
    d_pool = torch.from_numpy(np.ascontiguousarray(parena)).to(dev)
    d_arena = torch.zeros(reps * plen + 1024, dtype=torch.uint8, device=dev)
    for k in range(reps):
        d_arena[k * plen:k * plen + len(parena)].copy_(d_pool)
    del d_pool
    d_reqs = torch.from_numpy(reqs.view(np.uint8).reshape(-1)).to(dev)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    cap = n // 4 + (1 << 20)
    d_hits = torch.empty(cap, dtype=torch.int32, device=dev)
    e = engine.Engine(0)
    e.load(gblob, 1)
    s = torch.cuda.current_stream()
    e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), arena_len, n, d_out.data_ptr(), d_hits.data_ptr(), cap,
                s.cuda_stream)
    e.sync(s.cuda_stream)
    total = e.stats()["last_hits"]
    v = d_out.cpu().numpy().view(records.VERDICT_DTYPE)
    h = d_hits[:total].cpu().numpy().view(np.uint32)
    pool_n = len(preqs)
    per = total // reps
    assert per * reps == total and per > 5000
    v0 = v[:pool_n]
    for k in range(1, reps):
        vk = v[k * pool_n:(k + 1) * pool_n].copy()
        has = vk["n_hits"] > 0
        assert np.array_equal(vk["first_hit_off"][has] - k * per, v0["first_hit_off"][has])
        vk["first_hit_off"] = v0["first_hit_off"]
        assert vk.tobytes() == v0.tobytes(), f"replica {k} verdicts differ"
        assert np.array_equal(h[k * per:(k + 1) * per], h[:per]), f"replica {k} hit ids differ"
    m = 200_000
    exp, eh = Oracle(gblob, 1).match(preqs[:m], parena, nthreads=16, hit_cap=8 * m + 1024)
    got = v0[:m].copy()
    nh = int(got["n_hits"].sum())
    assert_verdicts_equal(got, exp, h[:nh], eh, "benched C4 pool")
    assert (exp["action"] == 6).sum() > 1000


def _batch(seed, n):
    ss = workloads.c4_sigset(800, 200)
    reqs, arena = records.gen_c4(n, ss, seed=seed, plant_rate=0.05, pool_mb=8)
    return workloads.c4_blob(ss, "block"), reqs, arena


def test_async_two_streams_two_threads(torch_dev):
    """gm_match_batch returns before its batch completes, and two batches enqueued from two
    threads on two streams of one ctx each match the oracle."""
    torch, dev = torch_dev
    ss = workloads.c4_sigset(800, 200)
    blob = workloads.c4_blob(ss, "block")
    batches = []
    for seed in (101, 202):
        reqs, arena = records.gen_c4(150_000, ss, seed=seed, plant_rate=0.05, pool_mb=8)
        batches.append((reqs, arena))
    e = engine.Engine(0)
    e.load(blob, 4)
    e.sync(0)
    streams = [torch.cuda.Stream(device=dev) for _ in batches]
    bufs = []
    for (reqs, arena) in batches:
        d_reqs, d_arena = _to_dev(torch, dev, reqs, arena)
        n = len(reqs)
        bufs.append((d_reqs, d_arena, len(arena), n, torch.empty(n * 32, dtype=torch.uint8, device=dev),
                     torch.empty(4 * n + 1024, dtype=torch.int32, device=dev)))
    torch.cuda.synchronize()
    pending = [None, None]

    def enqueue(k):
        d_reqs, d_arena, alen, n, d_out, d_hits = bufs[k]
        e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), alen, n, d_out.data_ptr(), d_hits.data_ptr(),
                    d_hits.numel(), streams[k].cuda_stream)
        pending[k] = not streams[k].query()   # still running when the call returned

    # warm the per-stream scratch (first batches on a stream allocate it)
    for k in range(2):
        enqueue(k)
        e.sync(streams[k].cuda_stream)
    th = [threading.Thread(target=enqueue, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert any(pending), "gm_match_batch waited for the device"
    oracle = Oracle(blob, 4)
    for k, (reqs, arena) in enumerate(batches):
        e.sync(streams[k].cuda_stream)
        total = e.stats()["last_hits"]
        d_reqs, d_arena, alen, n, d_out, d_hits = bufs[k]
        got = d_out.cpu().numpy().view(records.VERDICT_DTYPE)
        gh = d_hits.cpu().numpy().view(np.uint32)
        exp, eh = oracle.match(reqs, arena)
        assert_verdicts_equal(got, exp, gh[:len(eh)], eh, f"stream {k}")
        assert int(got["n_hits"].sum()) == len(eh) and total == len(eh)


def test_counters_cumulative_and_allreduce_out_of_place(torch_dev):
    """Counters accumulate over batches; the RCCL reduction (1 rank here) is out of place, so
    calling it after every batch gives the true totals, never a doubled count."""
    ss = workloads.c4_sigset(400, 100)
    reqs, arena = records.gen_c4(20_000, ss, plant_rate=0.1, pool_mb=4)
    b = workloads.c4_blob(ss, "monitoring")
    e = engine.Engine(0)
    e.load(b, 3)
    e.comm_init(engine.Engine.comm_unique_id(), 1, 0)
    got, gh = e.match_host(reqs, arena)
    st = e.stats()
    nl = st["n_locations"]
    loc = got["location_id"][got["location_id"] != 0xFFFFFFFF]
    one = np.concatenate([np.bincount(loc, minlength=nl), np.bincount(gh, minlength=st["n_sigs"])]).astype(np.uint64)
    for k in (1, 2, 3):
        if k > 1:
            e.match_host(reqs, arena)
        e.counters_allreduce(0)
        e.sync(0)
        assert np.array_equal(e.counters(), k * one)
        assert np.array_equal(e.counters_global(), k * one)
        e.counters_allreduce(0)   # a second reduction of the same state changes nothing
        assert np.array_equal(e.counters_global(), k * one)


def test_normalize_after_overflow_syncs_clean(torch_dev):
    """A normalisation enqueued after an overflowing batch completes with GM_OK (its own status)."""
    torch, dev = torch_dev
    ss = workloads.c4_sigset(200, 50)
    reqs, arena = records.gen_c4(5_000, ss, plant_rate=0.5, pool_mb=4)
    e = engine.Engine(0)
    e.load(workloads.c4_blob(ss), 3)
    with pytest.raises(engine.GmError) as ei:
        e.match_host(reqs, arena, hit_cap=10)
    assert ei.value.code == engine.GM_E_OVERFLOW
    paths = [b"/a/./b/../c", b"//x//y", b"/%41%2f"]
    buf = b"".join(p.ljust(16, b"\0") for p in paths)
    d_a = torch.from_numpy(np.frombuffer(buf, np.uint8).copy()).to(dev)
    d_off = torch.tensor([16 * i for i in range(len(paths))], dtype=torch.int64, device=dev)
    d_len = torch.tensor([len(p) for p in paths], dtype=torch.int32, device=dev)
    d_ol = torch.zeros(len(paths), dtype=torch.int32, device=dev)
    e.normalize_uris_ptr(d_a.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(paths), d_a.data_ptr(),
                         d_ol.data_ptr(), 0)
    e.sync(0)
    out = d_a.cpu().numpy().tobytes()
    ol = d_ol.cpu().numpy()
    assert [out[16 * i:16 * i + int(ol[i])] for i in range(len(paths))] == [b"/a/c", b"/x/y", b"/A/"]


# ---------------------------------------------------------------- counters: whole batches only
# a batch's location and rule hits accumulate in per-batch scratch and are committed
# by k_ctr_commit only when the batch is whole -- a void batch (hit_cap too small) adds nothing, so
# the caller's retry counts each request once (internal/metrics/collectors/manager.go:27-59).
def _one_batch_counters(e, got, gh):
    st = e.stats()
    nl = st["n_locations"]
    loc = got["location_id"][got["location_id"] != 0xFFFFFFFF]
    return np.concatenate([np.bincount(loc, minlength=nl),
                           np.bincount(gh, minlength=st["n_sigs"])]).astype(np.uint64)


def test_void_batch_commits_no_counters(torch_dev):
    ss = workloads.c4_sigset(400, 100)
    reqs, arena = records.gen_c4(20_000, ss, plant_rate=0.3, pool_mb=4)
    b = workloads.c4_blob(ss, "monitoring")
    e = engine.Engine(0)
    e.load(b, 3)
    for _ in range(2):   # the overflowing call, twice: nothing committed
        with pytest.raises(engine.GmError) as ei:
            e.match_host(reqs, arena, hit_cap=10)
        assert ei.value.code == engine.GM_E_OVERFLOW
        assert not e.counters().any()
    got, gh = e.match_host(reqs, arena)   # the retry with room: one batch's counts
    assert len(gh) > 10
    assert np.array_equal(e.counters(), _one_batch_counters(e, got, gh))
    exp, eh = Oracle(b, 3).match(reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "retry after a void batch")


@pytest.mark.parametrize("host,spill", [(True, True), (False, True), (True, False), (False, False)])
def test_set_overflow_continuation(torch_dev, host, spill):
    """a dedupe-set overflow (OV_SET: more unique hits + regex jobs than the set holds
    -- an attack burst) neither voids the batch nor re-runs it whole.  With the set shrunk
    (GM_CREATE_SET_SHIFT) the first pass overflows it: the pairs it refuses go to the spill, and
    gm_sync emits each distinct one (spill); with the spill shrunk too (GM_CREATE_SPILL_SHIFT) it
    overflows as well, and gm_sync redoes the requests it
    missed as a sub-batch with a set twice as large.  Either way GM_OK: verdicts and hits equal the
    oracle's, and the counters hold exactly one batch."""
    torch, dev = torch_dev
    ss, b = workloads.c4_stress_generation()
    reqs, arena = records.gen_c4(6_000, ss, seed=workloads.C4_STRESS_POOL_SEED + 9, plant_rate=0.3, stress=True)
    probe = engine.Engine(0)
    probe.load(b, 5)
    probe.match_host(reqs, arena)
    st = probe.stats()
    keys = st["last_pairs"] + st["last_jobs"]
    probe.close()
    assert keys > 2048, keys
    # the default set for 6000 requests holds 2^19 slots; shrink it below the keys but within
    # reach of the re-runs' doubling (x64 at most)
    shift = 1
    while (1 << 19) >> (shift + 1) >= keys // 2 and shift < 12:
        shift += 1
    e = engine.Engine(0, set_shift=shift, spill_shift=0 if spill else 8)
    e.load(b, 5)
    if host:
        got, gh = e.match_host(reqs, arena)   # no GmError
    else:
        d_reqs, d_arena = _to_dev(torch, dev, reqs, arena)
        n = len(reqs)
        d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        d_hits = torch.zeros(8 * n + 1024, dtype=torch.int32, device=dev)
        e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), len(arena), n, d_out.data_ptr(), d_hits.data_ptr(),
                    d_hits.numel(), 0)
        e.sync(0)
        got = d_out.cpu().numpy().view(records.VERDICT_DTYPE)
        gh = d_hits[:e.stats()["last_hits"]].cpu().numpy().view(np.uint32)
    st = e.stats()
    assert st["set_shift"] == shift, st
    if spill:
        assert st["last_spill"] > 0 and st["n_set_reruns"] == 0, st
    else:
        assert st["last_redo"] > 0 and st["n_set_reruns"] >= 1, st
    exp, eh = Oracle(b, 5).match(reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, f"set overflow continuation (shift {shift}, spill {spill})")
    assert np.array_equal(e.counters(), _one_batch_counters(e, got, gh))


# ---------------------------------------------------------------- internal overflow completes
# a batch that overflows an internal WAF buffer must complete on the device.  The
# scan's candidate regions and the context filter's survivor regions are finished by
# k_waf_direct; an overflowing pair or job list is replaced by the dedupe set (k_hits_scatter /
# k_waf_regex read it).  GM_CREATE_SCRATCH_SHIFT (a gm_create flag) shrinks the default capacities so
# that every continuation runs on a batch the oracle checks in seconds.
OV_PAIRS, OV_CAND, OV_SURV, OV_JOBS = 1, 4, 8, 128


def _engine_scaled(shift):
    e = engine.Engine(0, scratch_shift=shift)   # GM_CREATE_SCRATCH_SHIFT: buffers at 2^-shift
    return e


@pytest.mark.parametrize("scale,want", [(9, OV_CAND | OV_SURV), (12, OV_CAND | OV_SURV | OV_PAIRS)])
def test_internal_overflow_completes_on_device(torch_dev, scale, want):
    """The stress variant (many candidates, real matches) on a fresh stream with shrunken internal
    buffers: the first call returns GM_OK, the overflow bits show which continuations ran, and
    verdicts and hit ids equal the oracle's."""
    ss, b = workloads.c4_stress_generation()
    reqs, arena = records.gen_c4(6_000, ss, seed=workloads.C4_STRESS_POOL_SEED + 7, plant_rate=0.3, stress=True)
    e = _engine_scaled(scale)
    e.load(b, 5)
    got, gh = e.match_host(reqs, arena)          # no GmError: the batch completed
    ov = int(e.debug_status()[3])
    assert ov & want == want, f"overflow bits {ov:#x}, expected {want:#x} (continuations not exercised)"
    exp, eh = Oracle(b, 5).match(reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, f"overflow continuation (scale {scale})")


def test_always_match_list_overflow_redoes_requests(torch_dev):
    """The always-run slices' match list (k_waf_always_multi -> k_alw_emit) shrunk to 16 entries
    (GM_CREATE_SPILL_SHIFT(12)): the matches past it mark their requests, gm_sync redoes them as a
    sub-batch, and the batch -- GM_OK -- equals the oracle."""
    ss, b = workloads.c4_stress_generation()
    reqs, arena = records.gen_c4(6_000, ss, seed=workloads.C4_STRESS_POOL_SEED + 11, plant_rate=0.3, stress=True)
    e = engine.Engine(0, spill_shift=12)
    e.load(b, 5)
    got, gh = e.match_host(reqs, arena)          # no GmError
    st = e.stats()
    assert st["last_redo"] > 0, st               # the overflow was taken by the redo continuation
    exp, eh = Oracle(b, 5).match(reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "always-run match list overflow")


def test_job_list_overflow_runs_jobs_from_set(torch_dev):
    """Factor regexes that are not prefix-mode (k_waf_regex jobs) with a shrunken job list: the
    jobs run from the dedupe set and every hit equals the oracle's."""
    ss = workloads.c4_job_sigset()
    reqs, arena = records.gen_c4(8_000, ss, seed=records.SEED_BASE + 91, plant_rate=0.5, pool_mb=4)
    b = workloads.c4_blob(ss)
    e = _engine_scaled(12)
    e.load(b, 6)
    got, gh = e.match_host(reqs, arena)
    st = e.stats()
    ov = int(e.debug_status()[3])
    assert st["last_jobs"] > 0 and ov & OV_JOBS, f"jobs {st['last_jobs']}, overflow bits {ov:#x}"
    exp, eh = Oracle(b, 6).match(reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "job list overflow")


def test_stress_first_batch_default_sizing(torch_dev):
    """bench.py's stress leg at default sizing on a fresh stream: its first batch (which used to
    be void) returns GM_OK and equals the same batch run again once the stream's buffers grew."""
    torch, dev = torch_dev
    ss, b = workloads.c4_stress_generation()
    preqs, parena = records.gen_c4(200_000, ss, seed=workloads.C4_STRESS_POOL_SEED, stress=True, pool_mb=8)
    n = 2_000_000
    reqs, plen, reps, alen = workloads.replicate_pool(preqs, len(parena), n)
    d_pool = torch.from_numpy(np.ascontiguousarray(parena)).to(dev)
    d_arena = torch.zeros(reps * plen + 1024, dtype=torch.uint8, device=dev)
    for k in range(reps):
        d_arena[k * plen:k * plen + len(parena)].copy_(d_pool)
    d_reqs = torch.from_numpy(reqs.view(np.uint8).reshape(-1)).to(dev)
    cap = 4 * n + (1 << 20)
    outs = []
    e = engine.Engine(0)
    e.load(b, 2)
    s = torch.cuda.current_stream().cuda_stream
    ovs = []
    for _ in range(2):
        d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        d_hits = torch.zeros(cap, dtype=torch.int32, device=dev)
        e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), alen, n, d_out.data_ptr(), d_hits.data_ptr(), cap, s)
        e.sync(s)                                # GM_OK on the first call
        ovs.append(int(e.debug_status()[3]))
        tot = e.stats()["last_hits"]
        outs.append((d_out.cpu().numpy(), d_hits[:tot].cpu().numpy()))
    assert ovs[0] & (OV_CAND | OV_SURV), f"first batch did not overflow ({ovs[0]:#x}): the test lost its point"
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


def _set_shift_for(b, reqs, arena, slots_log2):
    """The GM_CREATE_SET_SHIFT that puts the default set (2^slots_log2 slots) below the batch's keys
    but within reach of the continuation's doubling."""
    probe = engine.Engine(0)
    probe.load(b, 5)
    probe.match_host(reqs, arena)
    st = probe.stats()
    keys = st["last_pairs"] + st["last_jobs"]
    probe.close()
    shift = 1
    while (1 << slots_log2) >> (shift + 1) >= keys // 2 and shift < 14:
        shift += 1
    return shift, keys


def test_set_overflow_continuation_cost(torch_dev):
    """The continuation's cost: a 200k-request stress batch whose set overflows completes in
    gm_sync in under 2x the time of the same batch on a context whose set fits (the sub-batch holds
    only the requests with a refused insert), with the same verdicts and hits, and one batch's
    counters.  Both are a fresh stream's first batch of this traffic (so both grow their candidate
    buffers on the device's continuation path), after a warm-up batch of the same shape without
    hits (buffers allocated)."""
    import time
    torch, dev = torch_dev
    ss, b = workloads.c4_stress_generation()
    reqs, arena = records.gen_c4(200_000, ss, seed=workloads.C4_STRESS_POOL_SEED + 11, stress=True, pool_mb=8)
    n = len(reqs)
    d_reqs, d_arena = _to_dev(torch, dev, reqs, arena)
    zero = torch.zeros_like(d_arena)
    cap = 8 * n + (1 << 16)
    # default set for 200k requests: 2 * (3 * 200k + 131072) -> 2^21 slots
    shift, keys = _set_shift_for(b, reqs, arena, 21)

    def first_batch(set_shift):
        e = engine.Engine(0, set_shift=set_shift)
        e.load(b, 5)
        d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        d_hits = torch.zeros(cap, dtype=torch.int32, device=dev)
        e.match_ptr(d_reqs.data_ptr(), zero.data_ptr(), len(arena), n, d_out.data_ptr(), d_hits.data_ptr(), cap, 0)
        e.sync(0)
        base = e.counters()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), len(arena), n, d_out.data_ptr(), d_hits.data_ptr(), cap, 0)
        e.sync(0)
        t = time.perf_counter() - t0
        st = e.stats()
        v = d_out.cpu().numpy().view(records.VERDICT_DTYPE).copy()
        h = d_hits[:st["last_hits"]].cpu().numpy().view(np.uint32).copy()
        ctr = e.counters() - base
        e.close()
        return v, h, ctr, t, st

    clean = [first_batch(0) for _ in range(3)]
    ref_v, ref_h, ref_c = clean[0][0], clean[0][1], clean[0][2]
    assert all(c[4]["n_set_reruns"] == 0 for c in clean)
    ov = [first_batch(shift) for _ in range(3)]
    for v, h, ctr, t, st in ov:
        assert st["last_spill"] > 0, (shift, keys, st)
        assert_verdicts_equal(v, ref_v, h, ref_h, f"continuation vs clean (shift {shift})")
        assert np.array_equal(ctr, ref_c)
    t_clean, t_ov = min(c[3] for c in clean), min(o[3] for o in ov)
    redo = [o[4]["last_spill"] for o in ov]
    print(f"continuation: {t_ov * 1e3:.2f} ms vs clean {t_clean * 1e3:.2f} ms; keys {keys}, set shift {shift}, "
          f"pairs spilled {redo} for {n} requests")
    assert t_ov < 2 * t_clean, (t_ov, t_clean, shift, keys, redo)


def test_two_batches_before_one_sync(torch_dev):
    """several batches queued on one stream before gm_sync.  An earlier batch's overflow
    is not lost when a later batch starts: its dedupe-set overflow is completed (re-run whole, its
    scratch being reused), and its hit_cap overflow is reported by the sync, with its counters not
    committed while the clean batch's are."""
    torch, dev = torch_dev
    ss, b = workloads.c4_stress_generation()
    ra, aa = records.gen_c4(6_000, ss, seed=workloads.C4_STRESS_POOL_SEED + 9, plant_rate=0.3, stress=True)
    rb, ab = records.gen_c4(4_000, ss, seed=workloads.C4_STRESS_POOL_SEED + 13, plant_rate=0.1, stress=True)
    exp_a, eh_a = Oracle(b, 5).match(ra, aa)
    exp_b, eh_b = Oracle(b, 5).match(rb, ab)
    shift, _ = _set_shift_for(b, ra, aa, 19)

    def enqueue(e, reqs, arena, cap):
        d_reqs, d_arena = _to_dev(torch, dev, reqs, arena)
        d_out = torch.empty(len(reqs) * 32, dtype=torch.uint8, device=dev)
        d_hits = torch.zeros(max(cap, 1), dtype=torch.int32, device=dev)
        e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), len(arena), len(reqs), d_out.data_ptr(), d_hits.data_ptr(),
                    cap, 0)
        return d_reqs, d_arena, d_out, d_hits

    def read(bufs, n_hits_total):
        v = bufs[2].cpu().numpy().view(records.VERDICT_DTYPE)
        return v, bufs[3][:n_hits_total].cpu().numpy().view(np.uint32)

    # A overflows its set, B is clean: one sync completes both
    e = engine.Engine(0, set_shift=shift)
    e.load(b, 5)
    A = enqueue(e, ra, aa, 8 * len(ra) + 1024)
    B = enqueue(e, rb, ab, 8 * len(rb) + 1024)
    e.sync(0)
    assert e.stats()["n_set_reruns"] >= 1   # A (not the stream's last batch) re-ran whole
    got_a, gh_a = read(A, int(len(eh_a)))
    got_b, gh_b = read(B, int(len(eh_b)))
    assert_verdicts_equal(got_a, exp_a, gh_a, eh_a, "queued batch A (set overflow)")
    assert_verdicts_equal(got_b, exp_b, gh_b, eh_b, "queued batch B")
    assert np.array_equal(e.counters(), _one_batch_counters(e, got_a, gh_a) + _one_batch_counters(e, got_b, gh_b))
    e.close()
    # A overflows hit_cap, B is clean: the sync reports the overflow; only B is counted
    e = engine.Engine(0)
    e.load(b, 5)
    A = enqueue(e, ra, aa, 10)
    B = enqueue(e, rb, ab, 8 * len(rb) + 1024)
    with pytest.raises(engine.GmError) as ei:
        e.sync(0)
    assert ei.value.code == engine.GM_E_OVERFLOW
    got_b, gh_b = read(B, int(len(eh_b)))
    assert_verdicts_equal(got_b, exp_b, gh_b, eh_b, "queued batch B after a void A")
    assert np.array_equal(e.counters(), _one_batch_counters(e, got_b, gh_b))
    e.close()
    # the same, through gm_sync_batches: the void batch is named (B, A, B: only the middle one)
    e = engine.Engine(0)
    e.load(b, 5)
    B1 = enqueue(e, rb, ab, 8 * len(rb) + 1024)
    A = enqueue(e, ra, aa, 10)
    B2 = enqueue(e, rb, ab, 8 * len(rb) + 1024)
    assert e.sync_batches(0) == [engine.GM_OK, engine.GM_E_OVERFLOW, engine.GM_OK]
    assert e.sync_batches(0) == []   # handed out once
    for bufs in (B1, B2):
        got_b, gh_b = read(bufs, int(len(eh_b)))
        assert_verdicts_equal(got_b, exp_b, gh_b, eh_b, "queued batch B beside a void A")
    assert np.array_equal(e.counters(), 2 * _one_batch_counters(e, got_b, gh_b))
    e.close()


def test_forced_sync_names_the_earlier_batch(torch_dev):
    """the 65th unsynced gm_match_batch completes the earlier 64 first; when one of them
    is void it answers GM_E_EARLIER (not the new batch's own outcome) and does not enqueue the new
    batch; gm_sync_batches then names the void one among the 64."""
    torch, dev = torch_dev
    ss, b = workloads.c4_stress_generation()
    r, a = records.gen_c4(64, ss, seed=workloads.C4_STRESS_POOL_SEED + 21, plant_rate=0.5, stress=True)
    exp, eh = Oracle(b, 5).match(r, a)
    assert len(eh) > 4
    e = engine.Engine(0)
    e.load(b, 5)
    d_reqs, d_arena = _to_dev(torch, dev, r, a)
    outs = [torch.empty(len(r) * 32, dtype=torch.uint8, device=dev) for _ in range(65)]
    hits = [torch.zeros(len(eh) + 1024, dtype=torch.int32, device=dev) for _ in range(65)]
    for i in range(64):
        cap = 2 if i == 7 else hits[i].numel()   # batch 7 overflows its hit_ids
        e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), len(a), len(r), outs[i].data_ptr(), hits[i].data_ptr(),
                    cap, 0)
    with pytest.raises(engine.GmError) as ei:
        e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), len(a), len(r), outs[64].data_ptr(), hits[64].data_ptr(),
                    hits[64].numel(), 0)
    assert ei.value.code == engine.GM_E_EARLIER
    st = e.sync_batches(0)
    assert len(st) == 64 and st[7] == engine.GM_E_OVERFLOW
    assert all(x == engine.GM_OK for i, x in enumerate(st) if i != 7)
    got = outs[63].cpu().numpy().view(records.VERDICT_DTYPE)
    assert_verdicts_equal(got, exp, hits[63][:len(eh)].cpu().numpy().view(np.uint32), eh, "batch 63")
    # 63 clean batches counted, the void one and the refused 65th not
    one = _one_batch_counters(e, got, hits[63][:len(eh)].cpu().numpy().view(np.uint32))
    assert np.array_equal(e.counters(), 63 * one)
    e.close()


GM_ROUTE_HELD = 0x80


@pytest.mark.parametrize("set_shift,spill_shift", [(None, 0), (0, 12), (None, 12)])
def test_held_verdicts_before_sync(torch_dev, set_shift, spill_shift):
    """a batch whose dedupe set (or spill, or always-run match list) overflowed is
    completed by gm_sync, but the documented chain match -> gm_select_peers -> gm_upstream_uris runs
    on the stream BEFORE gm_sync.  Every action the first pass can settle is final when its kernels
    end (a refused true hit blocks at once); a wallarm-block request whose hits only the continuation
    knows is marked GM_ROUTE_HELD with action PROXY, and the peer selection enqueued before gm_sync
    answers GM_PEER_DEFER for exactly those.  After gm_sync every verdict equals the oracle's and no
    HELD mark remains."""
    torch, dev = torch_dev
    ss, b = workloads.c4_stress_generation()
    reqs, arena = records.gen_c4(6_000, ss, seed=workloads.C4_STRESS_POOL_SEED + 9, plant_rate=0.3, stress=True)
    n = len(reqs)
    if set_shift is None:   # a set below the batch's unique keys (as test_set_overflow_continuation)
        probe = engine.Engine(0)
        probe.load(b, 5)
        probe.match_host(reqs, arena)
        st = probe.stats()
        keys = st["last_pairs"] + st["last_jobs"]
        probe.close()
        set_shift = 1
        while (1 << 19) >> (set_shift + 1) >= keys // 2 and set_shift < 12:
            set_shift += 1
    e = engine.Engine(0, set_shift=set_shift, spill_shift=spill_shift)
    e.load(b, 5)
    n_peers = e.stats()["n_peers"]
    state = torch.zeros(max(n_peers, 1) * 16, dtype=torch.uint8, device=dev)
    e.peers_init_ptr(state.data_ptr(), n_peers, 0)
    d_reqs, d_arena = _to_dev(torch, dev, reqs, arena)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_hits = torch.zeros(8 * n + 1024, dtype=torch.int32, device=dev)
    d_peer = torch.zeros(n, dtype=torch.int32, device=dev)
    e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), len(arena), n, d_out.data_ptr(), d_hits.data_ptr(),
                d_hits.numel(), 0)
    e.select_peers_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), len(arena), n, d_out.data_ptr(), state.data_ptr(),
                       n_peers, d_peer.data_ptr(), 0)
    torch.cuda.synchronize()   # the kernels are done; gm_sync has not run
    pre = d_out.cpu().numpy().view(records.VERDICT_DTYPE).copy()
    peer = d_peer.cpu().numpy().view(np.uint32).copy()
    e.sync(0)
    st = e.stats()
    assert st["last_spill"] > 0 or st["last_redo"] > 0, f"no set / spill overflow: the test exercises nothing {st}"
    got = d_out.cpu().numpy().view(records.VERDICT_DTYPE)
    gh = d_hits[:e.stats()["last_hits"]].cpu().numpy().view(np.uint32)
    exp, eh = Oracle(b, 5).match(reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, f"held batch (set shift {set_shift}, spill shift {spill_shift})")
    assert not (got["route_kind"] & GM_ROUTE_HELD).any(), "gm_sync left a HELD mark"
    held = (pre["route_kind"] & GM_ROUTE_HELD) != 0
    assert (pre["action"][held] == 0).all() and (pre["waf_mode"][held] == 3).all()
    assert (peer[held] == engine.GM_PEER_DEFER).all(), "a held request got a peer before gm_sync"
    # every other action was already final before gm_sync
    bad = np.nonzero(~held & (pre["action"] != exp["action"]))[0]
    assert len(bad) == 0, f"{len(bad)} requests changed action at gm_sync without a HELD mark, e.g. {bad[:5]}"
    if spill_shift == 12:
        assert held.any(), "the always-run list overflow marked no request HELD"
