"""Benches of the rows either side of the path (SURVEY.md §8 f), one GPU, inputs resident in HBM
before the timed region, HIP events on the launch stream around K calls:

  peers          gm_select_peers over 10M proxied verdicts of the peers workload (every LBMethod)
  peers-default  the same with every upstream on the reference's default "random two least_conn"
                 (config_params.go:123)
  wire           gm_parse_requests over synthetic HTTP/1.x messages (gpumatch.wire.synthetic)

Algorithmic bytes: peers = 32 B verdict + 64 B record + 4 B peer per request (+ the key bytes a
hash method reads, not counted); wire = message bytes + 80 B descriptor in, 64 B record + the
arena bytes out.  The CPU oracle is timed beside each on a bounded sample.

    python scripts/bench_next.py --what peers,peers-default,wire
"""

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


def timed(torch, fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s)
    for _ in range(steps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, e0.elapsed_time(e1) / steps


def bench_peers(torch, args, method):
    from gpumatch import engine, peers, records
    from oracle_py import Balancer, Oracle
    dev = torch.device("cuda", 0)
    b = peers.peers_blob(method)
    preqs, parena = peers.gen_requests(args.pool, seed=records.SEED_BASE + 70)
    n = args.requests
    pool_n = len(preqs)
    plen = (len(parena) + 15) & ~15
    reps = (n + pool_n - 1) // pool_n
    reqs = np.tile(preqs, reps)[:n]
    reqs["base"] += (np.repeat(np.arange(reps, dtype=np.uint64), pool_n)[:n] * np.uint64(plen))
    d_pool = torch.from_numpy(np.ascontiguousarray(parena)).to(dev)
    d_arena = torch.zeros(reps * plen + 1024, dtype=torch.uint8, device=dev)
    for k in range(reps):
        d_arena[k * plen:k * plen + len(parena)].copy_(d_pool)
    alen = reps * plen
    d_reqs = torch.from_numpy(reqs.view(np.uint8).reshape(-1)).to(dev)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_hits = torch.empty(1 << 16, dtype=torch.int32, device=dev)
    d_peer = torch.empty(n, dtype=torch.int32, device=dev)
    e = engine.Engine(0)
    e.load(b, 1)
    npeers = e.stats()["n_peers"]
    d_state = torch.zeros(npeers * 16, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    e.peers_init_ptr(d_state.data_ptr(), npeers, s)
    e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), alen, n, d_out.data_ptr(), d_hits.data_ptr(), 1 << 16, s)
    e.sync(s)

    def step():
        e.select_peers_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), alen, n, d_out.data_ptr(), d_state.data_ptr(),
                           npeers, d_peer.data_ptr(), s)
    wall_ms, ev_ms = timed(torch, step, args.steps, args.warmup)
    v = d_out[:pool_n * 32].cpu().numpy().view(records.VERDICT_DTYPE)
    proxied = float(np.mean(v["action"] == 0))
    # CPU: the oracle's balancers, one thread (sequential by nature), on a bounded sample
    o = Oracle(b, 1)
    bal = Balancer(o)
    m = min(pool_n, args.cpu_sample)
    t = time.perf_counter(); bal.select(preqs[:m], parena, v[:m]); cdt = time.perf_counter() - t
    alg = n * (32 + 64 + 4)
    print(json.dumps({
        "metric": "peer selections/sec", "value": n / (ev_ms * 1e-3), "unit": "requests/s",
        "config": {"workload": f"{'LBMethod ' + method if method else 'every LBMethod'}: "
                               f"{len(peers.UPSTREAMS) + 1} upstreams, {npeers} peers", "requests": n,
                   "proxied_fraction": round(proxied, 3)},
        "ms_per_call": ev_ms, "wall_ms_per_call": wall_ms,
        "algorithmic_GBps": alg / (ev_ms * 1e-3) / 1e9, "hbm_frac": alg / (ev_ms * 1e-3) / 8e12,
        "cpu_baseline": {"value": m / cdt, "unit": "requests/s", "cores": 1, "kind": "port",
                         "sample": f"first {m} verdicts of the pool ({cdt:.2f}s)"}}), flush=True)


def bench_wire(torch, args):
    from gpumatch import engine, wire
    from oracle_py import parse_requests
    dev = torch.device("cuda", 0)
    msgs_l, conn = wire.synthetic(args.wire_pool)
    pw, pm = wire.build(msgs_l, conn, align=1)
    reps = max(1, args.wire_requests // len(pm))
    n = reps * len(pm)
    msgs = np.tile(pm, reps)
    msgs["off"] += np.repeat(np.arange(reps, dtype=np.uint64), len(pm)) * np.uint64(len(pw))
    wbytes = np.tile(pw, reps)
    cap = wire.arena_bound(msgs)
    d_w = torch.from_numpy(wbytes).to(dev)
    d_m = torch.from_numpy(msgs.view(np.uint8).reshape(-1)).to(dev)
    d_reqs = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    d_arena = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_len = torch.zeros(1, dtype=torch.int64, device=dev)
    e = engine.Engine(0)
    s = torch.cuda.current_stream().cuda_stream

    def step():
        e.parse_ptr(d_w.data_ptr(), d_m.data_ptr(), n, d_reqs.data_ptr(), d_arena.data_ptr(), cap,
                    d_len.data_ptr(), s)
    wall_ms, ev_ms = timed(torch, step, args.steps, args.warmup)
    e.sync(s)
    out_bytes = int(d_len.item())
    alg = len(wbytes) + 80 * n + 64 * n + out_bytes
    m = min(len(pm), args.cpu_sample)
    t = time.perf_counter(); parse_requests(pw, pm[:m]); cdt = time.perf_counter() - t
    print(json.dumps({
        "metric": "requests parsed/sec", "value": n / (ev_ms * 1e-3), "unit": "requests/s",
        "config": {"workload": f"synthetic HTTP/1.x mix (gpumatch.wire.synthetic, {len(pm)} messages x {reps})",
                   "requests": n, "wire_bytes": int(len(wbytes))},
        "ms_per_call": ev_ms, "wall_ms_per_call": wall_ms,
        "algorithmic_GBps": alg / (ev_ms * 1e-3) / 1e9, "hbm_frac": alg / (ev_ms * 1e-3) / 8e12,
        "cpu_baseline": {"value": m / cdt, "unit": "requests/s", "cores": 1, "kind": "port",
                         "sample": f"first {m} messages ({cdt:.2f}s)"}}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="peers,peers-default,wire")
    ap.add_argument("--requests", type=int, default=10_000_000)
    ap.add_argument("--pool", type=int, default=200_000)
    ap.add_argument("--wire-requests", type=int, default=2_000_000)
    ap.add_argument("--wire-pool", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-sample", type=int, default=200_000)
    args = ap.parse_args()
    import torch
    for w in args.what.split(","):
        if w == "peers":
            bench_peers(torch, args, None)
        elif w == "peers-default":
            bench_peers(torch, args, "random two least_conn")
        elif w == "wire":
            bench_wire(torch, args)
        else:
            raise SystemExit(f"unknown bench {w}")


if __name__ == "__main__":
    main()
