"""GPU box debug: gm_parse_requests records vs the oracle's, per message (first mismatches)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from gpumatch import engine, records, wire  # noqa: E402
from oracle_py import parse_requests  # noqa: E402

n_syn = int(sys.argv[1]) if len(sys.argv) > 1 else 200
msgs, conn = wire.synthetic(n_syn, seed=99)
msgs = list(wire._EDGE) + msgs
conn = [{"https": False, "port": 80}] * len(wire._EDGE) + conn
W, M = wire.build(msgs, conn)
dev = torch.device("cuda", 0)
e = engine.Engine(0)
n = len(M)
cap = wire.arena_bound(M) * 8
d_w = torch.from_numpy(W).to(dev)
d_m = torch.from_numpy(M.view(np.uint8).reshape(-1).copy()).to(dev)
d_r = torch.zeros(n * 64 + 16, dtype=torch.uint8, device=dev)
d_a = torch.zeros(cap + 64, dtype=torch.uint8, device=dev)
d_len = torch.zeros(1, dtype=torch.int64, device=dev)
e.parse_ptr(d_w.data_ptr(), d_m.data_ptr(), n, d_r.data_ptr(), d_a.data_ptr(), cap, d_len.data_ptr(), 0)
try:
    e.sync(0)
except engine.GmError as x:
    print("sync:", x)
got = d_r[:n * 64].cpu().numpy().view(records.REQ_DTYPE)
import ctypes  # noqa: E402
L = engine.lib()
L.gm_debug_wire_sizes.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
sizes = np.zeros(n + 1, np.uint64)
L.gm_debug_wire_sizes(e.h, None, sizes.ctypes.data, n + 1)
print("sizes[:40]", sizes[:40].tolist())
print("arena_len", int(d_len.item()), "bound", wire.arena_bound(M))
exp, ea = parse_requests(W, M)
print("oracle arena", len(ea))
slots = np.diff(np.append(got["base"].astype(np.int64), int(d_len.item())))
shown = 0
for i in range(n):
    g, x = got[i], exp[i]
    keys = ("flags", "uri_len", "args_len", "hdr_len", "body_len", "host_len", "method_len", "ruri_len", "raddr_len")
    if any(int(g[k]) != int(x[k]) for k in keys) or list(g["pad0"]) != list(x["pad0"]):
        print(i, "slot", int(slots[i]), msgs[i][:100])
        print("   gpu", {k: int(g[k]) for k in keys}, list(g["pad0"]))
        print("   orc", {k: int(x[k]) for k in keys}, list(x["pad0"]))
        shown += 1
        if shown > 12:
            break
print("max slot", int(slots.max()), "at", int(np.argmax(slots)))
