"""Measurement: always-run slice match counts on the stress leg (exp build with GM_EXP_ALW_COUNT):
python scripts/alw_count.py [requests] -- prints status words 30 (wave steps with a match) and 31
(lanes with a match) of one batch."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gpumatch import engine, records, workloads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
ss, b = workloads.c4_stress_generation()
e = engine.Engine(0)
e.load(b, 2)
reqs, arena = records.gen_c4(n, ss, seed=workloads.C4_STRESS_POOL_SEED, stress=True, pool_mb=8)
dev = torch.device("cuda", 0)
d_r = torch.from_numpy(reqs.view(np.uint8).reshape(-1)).to(dev)
d_a = torch.from_numpy(np.ascontiguousarray(arena)).to(dev)
d_o = torch.empty(n * 32, dtype=torch.uint8, device=dev)
d_h = torch.empty(4 * n + (1 << 20), dtype=torch.int32, device=dev)
for _ in range(2):
    e.match_ptr(d_r.data_ptr(), d_a.data_ptr(), len(arena), n, d_o.data_ptr(), d_h.data_ptr(), d_h.numel(), 0)
    e.sync(0)
L = engine.lib()
L.gm_debug_status.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t]
st = (ctypes.c_uint32 * 64)()
L.gm_debug_status(e.h, st, 64)
print({"requests": n, "wave_steps_with_match": st[30], "lanes_with_match": st[31], "pairs": st[1], "hits": st[4]})
