"""Secondary benches: the routing configs C1 (cafe Ingress), C2 (advanced-routing VS + split),
C3 (1k regex locations) and C5 (mergeable, 1k hosts) at 10M requests on one GPU, requests
resident in HBM before the timed region, the CPU oracle timed on a bounded sample beside it.
The headline line (C4) is bench.py's; these are the other BASELINE.json configs.

    python scripts/bench_config.py --config c3 [--requests R] [--pool P] [--steps K] [--warmup W]

Prints one JSON line per config (requests/s, route kernel ms from HIP events, algorithmic
bytes per request after SURVEY.md §8(d), cpu_baseline)."""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def workload(cfg, pool):
    from gpumatch import records, workloads
    if cfg == "c1":
        return workloads.c1_blob(), records.gen_c1(pool), "C1: cafe Ingress host + prefix routing"
    if cfg == "c2":
        return workloads.c2_blob(), records.gen_c2(pool), \
            "C2: advanced-routing VS (header/cookie/arg/method rules) + 90/10 split + e2e complex VS"
    if cfg == "c3":
        regs = workloads.c3_regexes()
        return workloads.c3_blob(regs), workloads.gen_c3(pool, regs), \
            "C3: 1000 regex locations (RE2 subset, 5% PCRE-only) over 32-256 B URIs, 40% crafted to hit"
    if cfg == "c5":
        return workloads.c5_blob(), workloads.gen_c5(pool), "C5: mergeable Ingresses, 1000 hosts, Zipf(1.1)"
    raise SystemExit(f"unknown config {cfg}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--requests", type=int, default=10_000_000)
    ap.add_argument("--pool", type=int, default=200_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import torch
    from gpumatch import engine, workloads
    from oracle_py import Oracle
    for cfg in args.config.split(","):
        blob, (preqs, parena), desc = workload(cfg, args.pool)
        eng = engine.Engine(0, profile=True)
        eng.load(blob, 1)
        pool_n = len(preqs)
        plen = (len(parena) + 15) & ~15
        reps = (args.requests + pool_n - 1) // pool_n
        n = args.requests
        reqs = np.tile(preqs, reps)[:n]
        reqs["base"] += (np.repeat(np.arange(reps, dtype=np.uint64), pool_n)[:n] * np.uint64(plen))
        dev = torch.device("cuda", 0)
        d_pool = torch.from_numpy(np.ascontiguousarray(parena)).to(dev)
        d_arena = torch.empty(reps * plen + 1024, dtype=torch.uint8, device=dev)
        for k in range(reps):
            d_arena[k * plen:k * plen + len(parena)].copy_(d_pool)
        arena_len = reps * plen
        d_reqs = torch.from_numpy(reqs.view(np.uint8).reshape(-1)).to(dev)
        d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        d_hits = torch.empty(1 << 20, dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream()

        def step():
            eng.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), arena_len, n, d_out.data_ptr(),
                          d_hits.data_ptr(), 1 << 20, stream.cuda_stream)
            eng.sync(stream.cuda_stream)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        ms = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
            ms.append(eng.stats()["last_ms_route"])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rt = float(np.mean(ms))
        try:
            import ctypes
            fn = ctypes.CDLL(engine.LIB_PATH).gm_exp_read
            ex = (ctypes.c_ulonglong * 8)()
            fn(ex)
            print("exp counters (steps+warmup)", list(ex), flush=True)
        except (AttributeError, OSError):
            pass
        # the per-config roofline: SURVEY §8(d)'s algorithmic bytes per request
        # (workloads.algorithmic_bytes) over the step's wall time and over the route kernel's
        alg = workloads.algorithmic_bytes(reqs, cfg)
        roof = {"algorithmic_bytes_per_step": alg, "algorithmic_GBps_step": alg * args.steps / dt / 1e9,
                "hbm_frac_step": alg * args.steps / dt / 1e9 / 8000.0,
                "algorithmic_GBps_route": alg / (rt * 1e-3) / 1e9, "hbm_frac_route": alg / (rt * 1e-3) / 1e9 / 8000.0}
        if args.no_cpu:
            print(json.dumps({"config": cfg, "requests": n, "ms_per_step": dt / args.steps * 1e3,
                              "route_kernel_ms": rt, "value": n * args.steps / dt, **roof}), flush=True)
            del d_arena, d_reqs, d_out, d_hits, d_pool, eng
            continue
        # CPU oracle on a bounded sample of the pool
        cores = min(os.cpu_count() or 1, 16)
        o = Oracle(blob, 1)
        t = time.perf_counter(); o.match(preqs[:500], parena, nthreads=cores)
        rate = 500 / (time.perf_counter() - t)
        m = int(min(pool_n, max(500, rate * args.cpu_seconds)))
        t = time.perf_counter(); o.match(preqs[:m], parena, nthreads=cores); cdt = time.perf_counter() - t
        print(json.dumps({
            "metric": f"requests/sec ({cfg.upper()})", "value": n * args.steps / dt, "unit": "requests/s",
            "n_gpus": 1, "steps": args.steps, "ms_per_step": dt / args.steps * 1e3,
            "route_kernel_ms": rt, "config": {"workload": desc, "requests": n, "pool": pool_n}, **roof,
            "cpu_baseline": {"value": m / cdt, "unit": "requests/s", "cores": cores, "kind": "port",
                             "sample": f"first {m} requests of the pool ({cdt:.1f}s)"}}), flush=True)
        del d_arena, d_reqs, d_out, d_hits, d_pool, eng


if __name__ == "__main__":
    main()
