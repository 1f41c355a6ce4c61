"""CPU: where the C4 scan's candidates come from (no GPU).  Loads the benched C4 generation in a
compile-only context, restates the scan's and the context filter's rules over a pool of C4 requests
(gm_debug_waf_prefilter / _prefilter2: the kernels' tables and hashes), and counts the candidate
windows, the stage-2 survivors and the exact key-window hits, with the keys that draw the most.

    python scripts/cand_sources.py [--pool N] [--top K]      (GM_LIB selects another build)
"""
import argparse
import collections
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd"))
from gpumatch import engine, records, workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=50_000)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    ss, gblob = workloads.c4_bench_generation()
    e = engine.Engine(0, compile_only=True)
    e.load(gblob, 1)
    L = engine.lib()
    for f in ("gm_debug_waf_keys", "gm_debug_waf_lits"):
        getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    for f in ("gm_debug_waf_prefilter", "gm_debug_waf_prefilter2"):
        getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        getattr(L, f).restype = ctypes.c_int64
    n = L.gm_debug_waf_keys(e.h, None, 0)
    keys = np.zeros(n, np.uint32)
    L.gm_debug_waf_keys(e.h, keys.ctypes.data, n)
    st = e.stats()
    reqs, arena = records.gen_c4(a.pool, ss, seed=workloads.C4_POOL_SEED)
    A = np.ascontiguousarray(arena)
    cap = len(A) // 2
    out = np.zeros(cap, np.uint64)
    nc = L.gm_debug_waf_prefilter(e.h, A.ctypes.data, len(A), out.ctypes.data, cap)
    cand = out[:nc].astype(np.int64)
    ns = L.gm_debug_waf_prefilter2(e.h, A.ctypes.data, len(A), None, 0)
    w = (A[:-3].astype(np.uint32) | (A[1:-2].astype(np.uint32) << 8) | (A[2:-1].astype(np.uint32) << 16)
         | (A[3:].astype(np.uint32) << 24)) | np.uint32(0x20202020)
    wc = w[cand[cand < len(w)]]
    hit = np.isin(wc, keys)
    print(f"keys {n} (bloom pk {st['bloom_pk']}, modelled fp {st['bloom_fp_ppm']} ppm); pool {a.pool} requests, "
          f"{len(A) / 1e6:.1f} MB")
    print(f"candidate windows {nc} ({nc / a.pool:.3f} per request): key-window hits {int(hit.sum())}, "
          f"Bloom false positives {int((~hit).sum())}; stage-2 survivors {ns} ({ns / a.pool:.4f} per request)")
    u, c = np.unique(wc[hit], return_counts=True)
    for i in np.argsort(-c)[:a.top]:
        print(f"  {int(u[i]).to_bytes(4, 'little')!r:16} {int(c[i]):7d}")


if __name__ == "__main__":
    main()
