"""Benchmark: BASELINE.json metric on config C4 (10k-rule WAF signature set over URI / args /
headers / <= 8 KB body), 10M requests per GPU, requests resident in HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--requests R] [--pool P] [--no-cpu]

N > 1 is launched by torch.distributed.run (one rank per GPU); requests shard with no data-path
collective (weak scaling: every rank classifies its own R requests); the per-location and
per-rule hit counters are all-reduced with RCCL over xGMI once per timed interval
(gm_counters_allreduce, after the last step).
A "step" = one gm_match_batch + gm_sync over the rank's R requests.  --inflight D (default 1):
with D > 1 batches are pipelined over D streams -- step k is enqueued on stream k % D and completed
by its gm_sync when that stream comes round again -- so a batch's tail overlaps the next batch's
scan, as a server handing the engine consecutive batches would run it; every step is still a whole
batch with its own verdicts and hits.  The default stays 1: overlapped launches stretch each
kernel's duration, and the roofline fraction is read from the scan's launch duration (DESIGN.md §6
has the D = 2 numbers).  Rank 0 prints one JSON line (config.inflight = D).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd"))

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def check_build(st, args):
    """Refuse a library built with measurement or tuning macros (gm_stats.build_flags: GM_BUILD_EXPERIMENT,
    GM_BUILD_TUNING) unless asked; such a build is an A/B variant, not the shipped pipeline."""
    if st["build_flags"] and not args.allow_nondefault_build:
        raise SystemExit(f"bench.py: the loaded libgpumatch.so is a non-default build (build_flags "
                         f"{st['build_flags']:#x}); rebuild it with `make` or pass --allow-nondefault-build")
    if st.get("scratch_scale", 1.0) != 1.0 or st.get("set_shift", 0):
        raise SystemExit(f"bench.py: scratch capacities are scaled ({st['scratch_scale']}): not the default context")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--requests", type=int, default=10_000_000)
    ap.add_argument("--pool", type=int, default=1_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--stress-requests", type=int, default=2_000_000,
                    help="the C4 stress variant's batch (0: skip); reported under the line's 'stress' key")
    ap.add_argument("--no-alone", action="store_true",
                    help="skip the scan-alone measurement (profiling runs: kernel stats of the pipeline only)")
    ap.add_argument("--serial", action="store_true",
                    help="measurement: the route stage alone before the scan (GM_CREATE_SERIAL)")
    ap.add_argument("--config", default="c4", choices=("c4", "c5"),
                    help="c4: the headline (default); c5: BASELINE configs[4], a request stream sharded "
                         "over the ranks with the hit counters all-reduced (--stream, --batch)")
    ap.add_argument("--stream", type=int, default=100_000_000, help="c5: requests in the whole stream")
    ap.add_argument("--batch", type=int, default=10_000_000, help="c5: requests per gm_match_batch")
    ap.add_argument("--inflight", type=int, default=1,
                    help="batches in flight: step k runs on stream k %% inflight, and its gm_sync waits until the "
                         "stream comes round again, so one batch's tail (context filter, exact check, hit "
                         "emission) overlaps the next batch's route and scan (1: one batch at a time)")
    ap.add_argument("--allow-nondefault-build", action="store_true",
                    help="measure a library built with measurement / tuning macros (gm_stats build_flags != 0); "
                         "the line is then marked \"build\": \"nondefault\" and is not a headline number")
    args = ap.parse_args()
    if args.config == "c5":
        return c5_main(args)

    import torch
    from gpumatch import engine, records, workloads

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    # ---- generation: C4 signature set on the cafe Ingress, wallarm mode block
    t0 = time.time()
    # benign traffic sample (disjoint seed) for the prefilter's key / hash choice (GM_ENTRY_SAMPLE)
    ss, gblob = workloads.c4_bench_generation()
    eng = engine.Engine(local, profile=True, serial=args.serial)
    eng.load(gblob, 1)
    st = eng.stats()
    check_build(st, args)
    log(f"[rank {rank}] generation: {st['n_sigs']} rules ({st['n_sig_literals']} lit, {st['n_sig_regex']} re), "
        f"table {st['table_bytes'] / 1e6:.1f} MB, compile+load {time.time() - t0:.1f}s")

    # ---- synthetic requests: a P-request pool, replicated to R requests in HBM
    t0 = time.time()
    pool_n = min(args.pool, args.requests)
    preqs, parena = records.gen_c4(pool_n, ss, seed=workloads.C4_POOL_SEED)
    n = args.requests
    reqs, plen, reps, arena_len = workloads.replicate_pool(preqs, len(parena), n)
    log(f"[rank {rank}] pool {pool_n} requests / {len(parena) / 1e9:.2f} GB generated in {time.time() - t0:.1f}s; "
        f"x{reps} -> {n} requests")
    dev = torch.device("cuda", local)
    d_pool = torch.from_numpy(np.ascontiguousarray(parena)).to(dev)
    d_arena = torch.zeros(reps * plen + 1024, dtype=torch.uint8, device=dev)
    for k in range(reps):
        d_arena[k * plen:k * plen + len(parena)].copy_(d_pool)
    del d_pool
    d_reqs = torch.from_numpy(reqs.view(np.uint8).reshape(-1)).to(dev)
    D = max(1, args.inflight)
    outs = [torch.empty(n * 32, dtype=torch.uint8, device=dev) for _ in range(D)]
    d_out = outs[0]
    hit_cap = n // 4 + (1 << 20)
    hitss = [torch.empty(hit_cap, dtype=torch.int32, device=dev) for _ in range(D)]
    d_hits = hitss[0]
    zone_bytes = int(reqs["uri_len"].sum() + reqs["args_len"].sum() + reqs["hdr_len"].sum() + reqs["body_len"].sum())
    alg_bytes_req = workloads.algorithmic_bytes(reqs, "c4")
    torch.cuda.synchronize()
    log(f"[rank {rank}] resident in HBM: arena {arena_len / 1e9:.2f} GB, scanned zones {zone_bytes / 1e9:.2f} GB")

    stream = torch.cuda.current_stream()
    # D streams, each with its own verdict / hit buffers (and, in the library, its own scratch):
    # batch k goes to stream k % D; its gm_sync runs when the stream comes round again (or at the
    # end), so the GPU always holds the next batch while one completes
    streams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(D - 1)]
    uid = None
    if world > 1:
        obj = [engine.Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        eng.comm_init(obj[0], world, rank)
    pending = [False] * D
    stage = {"scan": [], "route": [], "verify": [], "tail": []}

    def complete(j, record):
        if not pending[j]:
            return
        eng.sync(streams[j].cuda_stream)
        pending[j] = False
        if record:
            s = eng.stats()
            for key in stage:
                stage[key].append(s["last_ms_" + key])

    def step(k, record=False):
        j = k % D
        complete(j, record)
        eng.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), arena_len, n, outs[j].data_ptr(), hitss[j].data_ptr(),
                      hit_cap, streams[j].cuda_stream)
        pending[j] = True

    def drain(record=False):
        for j in range(D):
            complete(j, record)
        if world > 1:   # job-wide counter totals, once per interval (out of place: local counters stay cumulative)
            eng.counters_allreduce(stream.cuda_stream)
            eng.sync(stream.cuda_stream)

    for w in range(args.warmup):
        step(w)
        log(f"[rank {rank}] warmup {w + 1}/{args.warmup}")
    drain()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(k, record=True)
    drain(record=True)
    torch.cuda.synchronize()
    scan_ms, route_ms, verify_ms, tail_ms = stage["scan"], stage["route"], stage["verify"], stage["tail"]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    s = eng.stats()
    dbg = eng.debug_status()
    log(f"[rank {rank}] status words: records {dbg[5]}, anchored-DFA bytes {dbg[8]} (max/lane {dbg[9]}), "
        f"full literal matches {dbg[10]}")
    if dbg[40:48].any():   # GM_EXP_EXACT_CNT builds (measurement): the exact check's probe counts
        log(f"[rank {rank}] exact-check counts: survivors {dbg[45]}, bucket probes {dbg[40]} (max {dbg[41]}), "
            f"buckets hit {dbg[47]}, check-word rounds {dbg[42]} (max bucket {dbg[43]}), literal compares {dbg[44]}")
    log(f"[rank {rank}] {args.steps} steps in {elapsed:.3f}s; candidates {s['last_candidates']}, ctx-pass {s['last_ctx_pass']}, jobs {s['last_jobs']}, pairs "
        f"{s['last_pairs']}, hits {s['last_hits']}; ms route {np.mean(route_ms):.3f} scan {np.mean(scan_ms):.3f} "
        f"verify {np.mean(verify_ms):.3f} tail {np.mean(tail_ms):.3f}")

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    ms_step = elapsed / args.steps * 1e3
    total_reqs = n * world * args.steps
    scan_avg = float(np.mean(scan_ms))
    achieved = zone_bytes / (scan_avg * 1e-3) / 1e9
    result = {
        "metric": "requests/sec (10k-rule WAF signature set, C4)",
        "value": total_reqs / elapsed,
        "unit": "requests/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (numpy PCG64 seed 0xC0FFEE+3; 1M-request pool replicated in HBM)",
        "config": {"workload": "C4: 10k-rule WAF signature set (8000 literals + 2000 RE2-subset regexes) over "
                               "URI/args/headers/<=8KB body, cafe Ingress, wallarm_mode block",
                   "requests_per_gpu": n, "rules": int(st["n_sigs"]), "parallelism": f"dp{world} (request shards)",
                   "inflight": D},
        "scanned_GBps": (alg_bytes_req + 4 * int(s["last_hits"])) * world * args.steps / elapsed / 1e9,
        "hbm_frac_pipeline": (alg_bytes_req + 4 * int(s["last_hits"])) * world * args.steps / elapsed / 1e9
                             / HBM_PEAK_GBPS,
        "stage_ms": {"route": float(np.mean(route_ms)), "scan": scan_avg, "verify": float(np.mean(verify_ms)),
                     "tail": float(np.mean(tail_ms))},
        "roofline": {"bound": "hbm", "kernel": "k_waf_scan", "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                     "algorithmic_bytes_per_launch": zone_bytes},
    }
    result["roofline"].update(profiled(zone_bytes, st["csrc_hash"]))
    if st["build_flags"]:
        result["build"] = f"nondefault (build_flags {st['build_flags']:#x})"
    if world == 1 and not args.serial and not args.no_alone:
        # the scan kernel alone (GM_CREATE_SERIAL: the route first, then the scan on its own), on
        # the same resident batch: its own roofline fraction beside the in-pipeline one above,
        # where the route shares the CUs
        eng_s = engine.Engine(local, profile=True, serial=True)
        eng_s.load(gblob, 1)
        alone, alone_route = [], []
        for k in range(1 + 3):
            eng_s.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), arena_len, n, d_out.data_ptr(), d_hits.data_ptr(),
                            hit_cap, stream.cuda_stream)
            eng_s.sync(stream.cuda_stream)
            if k:
                alone.append(eng_s.stats()["last_ms_scan"])
                alone_route.append(eng_s.stats()["last_ms_route"])
        eng_s.close()
        a_ms = float(np.mean(alone))
        result["roofline"]["scan_alone_ms"] = a_ms
        result["stage_ms"]["route_alone"] = float(np.mean(alone_route))
        result["roofline"]["frac_alone"] = zone_bytes / (a_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
    if world == 1 and args.stress_requests > 0:
        del d_arena, d_reqs, d_out, d_hits
        torch.cuda.empty_cache()
        result["stress"] = stress_leg(torch, engine, records, workloads, args, local)
    if not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(ss, gblob, preqs, parena, args.cpu_seconds)
    if dist:
        dist.destroy_process_group()
    print(json.dumps(result), flush=True)


def c5_main(args):
    """BASELINE.json configs[4]: mergeable Ingresses (1k hosts, wildcard TLS), a --stream request
    stream sharded contiguously over WORLD_SIZE ranks (gpumatch.shard: the same slice / batch /
    reduce code tests/test_multi_cpu.py drives with gloo), each rank's slice resident in HBM and
    classified in --batch requests per gm_match_batch; after every step the per-location hit
    counters are all-reduced out of place with RCCL (gm_counters_allreduce).  Weak scaling is not
    this config's shape: the stream's size is fixed, so "scaling" is "strong"."""
    import torch
    from gpumatch import engine, shard, workloads
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    t0 = time.time()
    blob = workloads.c5_blob()
    eng = engine.Engine(local, profile=True)
    eng.load(blob, 1)
    check_build(eng.stats(), args)
    preqs, parena = workloads.gen_c5(min(args.pool, 200_000))
    lo, hi = shard.shard_bounds(args.stream, world, rank)
    reqs, plen, first, ncopies, alen = shard.stream_records(preqs, len(parena), lo, hi)
    n = hi - lo
    dev = torch.device("cuda", local)
    d_pool = torch.from_numpy(np.ascontiguousarray(parena)).to(dev)
    d_arena = torch.zeros(ncopies * plen + 1024, dtype=torch.uint8, device=dev)
    for k in range(ncopies):
        d_arena[k * plen:k * plen + len(parena)].copy_(d_pool)
    del d_pool
    d_reqs = torch.from_numpy(reqs.view(np.uint8).reshape(-1)).to(dev)
    d_out = torch.empty(max(n, 1) * 32, dtype=torch.uint8, device=dev)
    d_hits = torch.empty(1 << 16, dtype=torch.int32, device=dev)
    alg = workloads.algorithmic_bytes(reqs, "c5")
    torch.cuda.synchronize()
    log(f"[rank {rank}] C5: stream [{lo}, {hi}) of {args.stream}, {ncopies} pool copies ({alen / 1e9:.2f} GB) "
        f"resident; setup {time.time() - t0:.1f}s")
    obj = [engine.Engine.comm_unique_id() if rank == 0 else None]
    if dist:
        dist.broadcast_object_list(obj, src=0)
    eng.comm_init(obj[0], world, rank)
    stream = torch.cuda.current_stream().cuda_stream
    route_ms = []

    def classify(b0, b1):   # positions relative to this rank's slice
        eng.match_ptr(d_reqs.data_ptr() + 64 * b0, d_arena.data_ptr(), alen, b1 - b0, d_out.data_ptr() + 32 * b0,
                      d_hits.data_ptr(), 1 << 16, stream)

    def after_step(_step):
        eng.counters_allreduce(stream)   # job-wide totals, out of place
        eng.sync(stream)
        route_ms.append(eng.stats()["last_ms_route"])

    shard.run_stream(classify, 0, n, args.batch, after_step, steps=max(1, args.warmup))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    route_ms.clear()
    t_start = time.perf_counter()
    shard.run_stream(classify, 0, n, args.batch, after_step, steps=args.steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the reduced totals: every rank's locations, steps + warmup times the stream
    tot = eng.counters_global()
    st = eng.stats()
    routed = int(tot[:st["n_locations"]].sum())
    log(f"[rank {rank}] {args.steps} steps in {elapsed:.3f}s; job-wide location hits {routed}")
    if rank == 0:
        print(json.dumps({
            "metric": "requests/sec (C5: mergeable Ingresses, 1k hosts incl. wildcard TLS, request stream sharded "
                      "over the GPUs, hit-counter all-reduce)",
            "value": args.stream * args.steps / elapsed, "unit": "requests/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (workloads.gen_c5 pool, Zipf(1.1) hosts, replicated into the stream)",
            "config": {"workload": "C5: mergeable Ingresses, 1000 hosts x 1-8 minions, wildcard TLS",
                       "stream_requests": args.stream, "batch": args.batch,
                       "parallelism": f"dp{world} (contiguous stream shards, RCCL counter all-reduce)"},
            "route_ms_per_batch_last": float(np.mean(route_ms)) if route_ms else None,
            "algorithmic_GBps": alg * world * args.steps / elapsed / 1e9,
            "job_location_hits": routed}), flush=True)
    if dist:
        dist.destroy_process_group()


def stress_leg(torch, engine, records, workloads, args, local):
    """The C4 stress variant beside the headline: vocabulary literals that
    benign SQL / HTML text also speaks, 10% factorless regexes (k_waf_always on every (request,
    zone)) -- a 200k-request pool replicated to --stress-requests in HBM, K steps timed the same
    way.  Not the headline: the headline config stays C4."""
    ss, b = workloads.c4_stress_generation()
    e = engine.Engine(local, profile=True)
    e.load(b, 2)
    n = args.stress_requests
    preqs, parena = records.gen_c4(min(200_000, n), ss, seed=workloads.C4_STRESS_POOL_SEED, stress=True, pool_mb=8)
    reqs, plen, reps, alen = workloads.replicate_pool(preqs, len(parena), n)
    dev = torch.device("cuda", local)
    d_pool = torch.from_numpy(np.ascontiguousarray(parena)).to(dev)
    d_arena = torch.zeros(reps * plen + 1024, dtype=torch.uint8, device=dev)
    for k in range(reps):
        d_arena[k * plen:k * plen + len(parena)].copy_(d_pool)
    d_reqs = torch.from_numpy(reqs.view(np.uint8).reshape(-1)).to(dev)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    cap = 4 * n + (1 << 20)
    d_hits = torch.empty(cap, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def step():
        e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), alen, n, d_out.data_ptr(), d_hits.data_ptr(), cap, s)
        e.sync(s)
    steps = max(1, min(args.steps, 5))
    # warmup: a batch whose hits overflow d_hits returns GM_E_OVERFLOW with no counters committed and
    # grows the stream's buffers (gm_sync); the retry is a whole batch
    ok, tries = 0, 0
    while ok < max(1, args.warmup) and tries < 12:
        tries += 1
        try:
            step()
            ok += 1
        except engine.GmError as err:
            if err.code != engine.GM_E_OVERFLOW:
                raise
            log(f"[stress] warmup batch overflowed the stream's buffers (grown): {err}")
    torch.cuda.synchronize()
    ms = {"route": [], "scan": [], "verify": [], "tail": []}
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
        st = e.stats()
        for k in ms:
            ms[k].append(st["last_ms_" + k])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = e.stats()
    log(f"[stress] {steps} steps of {n} requests in {dt:.3f}s; candidates {st['last_candidates']}, ctx-pass "
        f"{st['last_ctx_pass']}, jobs {st['last_jobs']}, hits {st['last_hits']}")
    return {"workload": "C4 stress: 8000 vocabulary literals (no random tails) + 2000 regexes, 10% without a "
                        ">= 4-byte factor; benign text with SQL / HTML / shell vocabulary (gpumatch.sigs."
                        "gen_waf_sigset_stress, records.gen_c4(stress=True))",
            "requests": n, "value": n * steps / dt, "unit": "requests/s", "ms_per_step": dt / steps * 1e3,
            "candidates_per_request": st["last_candidates"] / n, "ctx_pass_per_request": st["last_ctx_pass"] / n,
            "jobs_per_request": st["last_jobs"] / n, "hits_per_request": st["last_hits"] / n,
            "always_regexes": int(st["n_sig_regex_always"]),
            "stage_ms": {k: float(np.mean(v)) for k, v in ms.items()}}


# The committed profiles of this bench's C4 scan (scripts/scan_profile.py over a rocprofv3
# --kernel-trace --stats run and the PMC passes of scripts/pmc.sh on the same tree), stamped with
# the hash of the kernel sources: profiles/*_scan_profile.json.  The one whose hash is the
# library's is used; none is used when no hash matches: a new kernel never pairs with an old
# profile (VERDICT r2 "Next round" 1).
SCAN_PROFILE_GLOB = "profiles/*_scan_profile.json"


def profiled(zone_bytes: int, lib_hash: str) -> dict:
    """roofline fields from the committed same-tree profile: `traffic` (HBM read bytes per
    k_waf_scan launch, 2 x FETCH_SIZE x 1024 per the gfx950 correction in MI355X_MICROARCH.md),
    the LDS bank-conflict rate of the Bloom probes (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE), and
    `frac_profiled` = zone bytes / the rocprofv3 average k_waf_scan duration / HBM peak.  Counters
    cannot be read inside the timed run, so these come from the profile, named with its source.
    The profile pairs with the LIBRARY benched: `lib_hash` is the source hash libgpumatch.so was
    built from (gm_stats_t.csrc_hash), so a stale prebuilt library never pairs with a profile of
    newer sources; `tree_hash` (the sources beside it) is reported for comparison."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from scan_profile import csrc_hash
    here = lib_hash
    tree = csrc_hash(ROOT)
    out = {"traffic": None, "frac_profiled": None, "csrc_hash": here, "tree_hash": tree,
           "anchor": "frac_profiled (rocprofv3 average of k_waf_scan; `frac` is the HIP-event time on this run)"}
    if here != tree:
        out["lib_status"] = f"library built from {here}, sources beside it hash {tree}"
    import glob
    found = []
    for path in sorted(glob.glob(os.path.join(ROOT, SCAN_PROFILE_GLOB)), key=os.path.getmtime):
        try:
            found.append((os.path.relpath(path, ROOT), json.load(open(path))))
        except (OSError, ValueError):
            continue
    if not found:
        out["profile_status"] = f"no profile ({SCAN_PROFILE_GLOB})"
        return out
    same = [(p, s) for p, s in found if s.get("csrc_hash") == here]
    if not same:
        p, s = found[-1]
        out["profile_status"] = (f"stale: no profile of the benched sources {here} (newest: {p}, "
                                 f"{s.get('csrc_hash')}); traffic and frac_profiled withheld")
        return out
    # (of several same-tree profiles, one with its PMC passes first, then the newest)
    p, s = sorted(same, key=lambda ps: ps[1].get("pmc_csrc_hash") == here)[-1]
    out["profile_source"] = p
    out["profile_status"] = "same tree"
    avg = s.get("k_waf_scan_avg_ns")
    if avg:
        out["scan_ms_profiled"] = avg / 1e6
        out["frac_profiled"] = zone_bytes / (avg * 1e-9) / 1e9 / HBM_PEAK_GBPS
    if s.get("pmc_csrc_hash") == here and s.get("k_waf_scan_hbm_read_bytes_per_launch") is not None:
        out["traffic"] = s["k_waf_scan_hbm_read_bytes_per_launch"]
        out["traffic_unit"] = "bytes/launch"
        out["traffic_source"] = f"{s.get('pmc_summary')} (rocprofv3 --pmc FETCH_SIZE, x2 gfx950)"
        if s.get("k_waf_scan_lds_bank_conflict_rate") is not None:
            out["lds_bank_conflict_rate"] = s["k_waf_scan_lds_bank_conflict_rate"]
    elif s.get("pmc_csrc_hash") != here:
        out["traffic_status"] = "PMC passes from other sources; traffic withheld"
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _host_threads():
    """The CPUs this process may run on (sched_getaffinity), bounded by the box's CPU share
    (OMP_NUM_THREADS: 16 per GPU on the bench pool; os.cpu_count() there is the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, share) if share > 0 else n)


def cpu_baseline(ss, gblob, preqs, parena, seconds):
    """A competent CPU engine on the same C4 requests: the oracle's C restatement (Aho-Corasick
    for the literals, PCRE 8.39 for the regexes) with every regex behind its required-literal
    prefilter (a second Aho-Corasick over the factors, oracle/gm_oracle.c orc_set_prefilter), on
    every host thread this process may use, plus a one-thread figure.  Bounded samples of the pool,
    ~seconds of wall time each."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import Oracle
    cores = _host_threads()
    o = Oracle(gblob, 1, prefilter=True)

    def rate(threads, secs):
        probe = 400
        t = time.perf_counter()
        o.match(preqs[:probe], parena, nthreads=threads)
        r0 = probe / (time.perf_counter() - t)
        m = int(min(len(preqs), max(probe, r0 * secs)))
        t = time.perf_counter()
        o.match(preqs[:m], parena, nthreads=threads)
        dt = time.perf_counter() - t
        return m / dt, m, dt
    v, m, dt = rate(cores, seconds)
    v1, m1, dt1 = rate(1, seconds / 3)
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return {"value": v, "unit": "requests/s", "cores": cores, "kind": "port",
            "value_1core": v1, "cores_1": 1, "cpu_model": _cpu_model(),
            # the box is one GPU's share of a larger host: os.cpu_count() is the whole machine,
            # OMP_NUM_THREADS the share this job may use; the line says which it ran on
            "host_cpus": os.cpu_count(), "affinity_cpus": aff,
            "cpu_share": os.environ.get("OMP_NUM_THREADS") or "unset",
            "per_core_value_x_host_cpus": v1 * (os.cpu_count() or 1),
            "engine": "oracle/gm_oracle.c: Aho-Corasick literals + PCRE 8.39 regexes behind a required-factor prefilter",
            "sample": f"first {m} requests of the C4 pool ({dt:.1f}s wall, {cores} threads); "
                      f"1-thread: first {m1} ({dt1:.1f}s)"}


if __name__ == "__main__":
    main()
