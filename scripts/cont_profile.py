"""Kernel trace of one dedupe-set continuation (measurement script): a 200k-request stress batch on
a context whose set is shrunk (GM_CREATE_SET_SHIFT) so that gm_sync redoes the requests with refused
inserts.  Run under `rocprofv3 --kernel-trace`; scripts/cont_trace.py prints the kernel sequence."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd"))
import numpy as np
import torch

from gpumatch import engine, records, workloads

shift = int(sys.argv[1]) if len(sys.argv) > 1 else 5
ss, b = workloads.c4_stress_generation()
reqs, arena = records.gen_c4(200_000, ss, seed=workloads.C4_STRESS_POOL_SEED + 11, stress=True, pool_mb=8)
dev = torch.device("cuda", 0)
n = len(reqs)
d_reqs = torch.from_numpy(np.ascontiguousarray(reqs).view(np.uint8).reshape(-1)).to(dev)
d_arena = torch.zeros(len(arena) + 1024, dtype=torch.uint8, device=dev)
d_arena[:len(arena)].copy_(torch.from_numpy(arena))
zero = torch.zeros_like(d_arena)
cap = 8 * n + (1 << 16)
d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
d_hits = torch.zeros(cap, dtype=torch.int32, device=dev)
for s in (0, shift):
    e = engine.Engine(0, set_shift=s)
    e.load(b, 5)
    for arr in (zero, d_arena):
        e.match_ptr(d_reqs.data_ptr(), arr.data_ptr(), len(arena), n, d_out.data_ptr(), d_hits.data_ptr(), cap, 0)
        e.sync(0)
    print("shift", s, "reruns", e.stats()["n_set_reruns"], "redo", e.stats()["last_redo"], flush=True)
    e.close()
