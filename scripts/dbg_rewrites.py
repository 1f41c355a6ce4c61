"""Debug: first differences of the parse -> match chain (GPU vs oracle) on the rewrites config."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
from gpumatch import engine, records, wire
from oracle_py import Oracle, parse_requests
from test_rewrites import KATS, cafe_rewrites_blob
from test_gpu_rewrites import _targets
dev = torch.device("cuda", 0)
b = cafe_rewrites_blob()
targets = [t.encode() for t, _ in KATS] + _targets(100_000, 31)
msgs = [b"GET " + t + b" HTTP/1.1\r\nHost: cafe.example.com\r\n\r\n" for t in targets]
w, m = wire.build(msgs, [{"https": False, "port": 80}] * len(msgs))
n = len(m)
oreqs, oarena = parse_requests(w, m)
o = Oracle(b, 1)
ov, _ = o.match(oreqs, oarena, nthreads=16)
e = engine.Engine(0); e.load(b, 1)
s = torch.cuda.current_stream().cuda_stream
d_w = torch.from_numpy(w).to(dev); d_m = torch.from_numpy(m.view(np.uint8).reshape(-1)).to(dev)
cap = wire.arena_bound(m)
d_reqs = torch.empty(n * 64, dtype=torch.uint8, device=dev); d_arena = torch.empty(cap + 1024, dtype=torch.uint8, device=dev)
d_alen = torch.zeros(1, dtype=torch.int64, device=dev); d_v = torch.empty(n * 32, dtype=torch.uint8, device=dev)
d_hits = torch.empty(1 << 16, dtype=torch.int32, device=dev)
e.parse_ptr(d_w.data_ptr(), d_m.data_ptr(), n, d_reqs.data_ptr(), d_arena.data_ptr(), cap, d_alen.data_ptr(), s)
e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), cap, n, d_v.data_ptr(), d_hits.data_ptr(), 1 << 16, s, arena_len_dev=d_alen.data_ptr())
e.sync(s)
gv = d_v.cpu().numpy().view(records.VERDICT_DTYPE)
greqs = d_reqs.cpu().numpy().view(records.REQ_DTYPE); garena = d_arena.cpu().numpy()
# matcher alone on the oracle's records
gv2, _ = e.match_host(oreqs, oarena)
bad = np.nonzero((gv["action"] != ov["action"]) | (gv["location_id"] != ov["location_id"]))[0]
bad2 = np.nonzero((gv2["action"] != ov["action"]) | (gv2["location_id"] != ov["location_id"]))[0]
print("chain mismatches", len(bad), "matcher-on-oracle-records mismatches", len(bad2))
for i in list(bad[:6]) + list(bad2[:6]):
    print("target", targets[i][:80])
    print("  gpu v", gv[i]); print("  gpu2 v", gv2[i]); print("  orc v", ov[i])
    for f in ("uri", "args", "host", "ruri"):
        print("  ", f, records.field_bytes(greqs, garena, i, f)[:60], records.field_bytes(oreqs, oarena, i, f)[:60])
    print("   flags", greqs[i]["flags"], oreqs[i]["flags"])
