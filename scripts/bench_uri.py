"""Bench of gm_normalize_uris ($uri normalisation) on one GPU.

10M synthetic raw paths (a 200k pool from tests/test_uri.random_paths, replicated in HBM),
resident before the timed region; HIP events around K launches on the launch stream.
Prints one JSON line: paths/s and algorithmic GB/s (input bytes + output bytes + 16 B per path).
"""

from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from gpumatch import engine  # noqa: E402
from test_uri import random_paths  # noqa: E402


def main(n_total=10_000_000, pool=200_000, steps=10, warmup=2):
    paths = random_paths(pool, 23)
    lens = np.array([len(p) for p in paths], np.uint32)
    reps = n_total // pool
    lens = np.tile(lens, reps)
    offs = np.zeros(len(lens), np.uint64)
    offs[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    arena = np.tile(np.frombuffer(b"".join(paths), np.uint8), reps)
    dev = torch.device("cuda:0")
    eng = engine.Engine(0)
    A = torch.from_numpy(arena).to(dev)
    O = torch.from_numpy(offs.view(np.int64)).to(dev)
    N = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty_like(A)
    ol = torch.empty(len(lens), dtype=torch.int32, device=dev)
    n = len(lens)
    for _ in range(warmup):
        eng.normalize_uris_ptr(A.data_ptr(), O.data_ptr(), N.data_ptr(), n, out.data_ptr(), ol.data_ptr())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        eng.normalize_uris_ptr(A.data_ptr(), O.data_ptr(), N.data_ptr(), n, out.data_ptr(), ol.data_ptr())
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / steps
    olen = ol.cpu().numpy().view(np.uint32)
    # CPU baseline: the oracle's batch restatement on one host thread over the first pool copy
    import ctypes
    from oracle_py import lib as orc_lib
    L = orc_lib()
    L.orc_normalize_batch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32] + [ctypes.c_void_p] * 2
    cpu_out = np.empty(int(offs[pool - 1]) + int(lens[pool - 1]), np.uint8)
    cpu_len = np.empty(pool, np.uint32)
    reps_cpu, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < 3.0:
        L.orc_normalize_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, pool, cpu_out.ctypes.data,
                              cpu_len.ctypes.data)
        reps_cpu += 1
    cpu_rate = reps_cpu * pool / (time.perf_counter() - t1)
    assert np.array_equal(cpu_len, olen[:pool]), "GPU and CPU oracle disagree"
    out_bytes = int(olen[olen != 0xFFFFFFFF].astype(np.uint64).sum())
    algo = int(lens.astype(np.uint64).sum()) + out_bytes + 16 * n
    print(json.dumps({"metric": "paths/sec ($uri normalisation)", "value": n / (ms * 1e-3), "unit": "paths/s",
                      "ms_per_launch": ms, "paths": n, "mean_len": float(lens.mean()),
                      "algorithmic_GBps": algo / (ms * 1e-3) / 1e9, "hbm_frac": algo / (ms * 1e-3) / 8e12,
                      "invalid_frac": float((olen == 0xFFFFFFFF).mean()), "wall_s": wall,
                      "cpu_baseline": {"value": cpu_rate, "unit": "paths/s", "cores": 1, "kind": "port",
                                       "sample": f"{reps_cpu} passes over the {pool}-path pool (~3 s)"}}))


if __name__ == "__main__":
    main()
