"""How many requests of a routing config take k_route's SLOW pass (batch status word 17):
python scripts/route_slow_count.py c2"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gpumatch import engine  # noqa: E402
import bench_config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
blob, (reqs, arena), _ = bench_config.workload(cfg, 200_000)
e = engine.Engine(0)
e.load(blob, 1)
dev = torch.device("cuda:0")
d_r = torch.from_numpy(reqs.view(np.uint8).copy()).to(dev)
d_a = torch.from_numpy(np.concatenate([arena, np.zeros(4096, np.uint8)])).to(dev)
n = len(reqs)
d_o = torch.empty(n * 32, dtype=torch.uint8, device=dev)
e.match_ptr(d_r.data_ptr(), d_a.data_ptr(), len(arena), n, d_o.data_ptr(), 0, 0, 0)
e.sync(0)
st = e.debug_status()
print(cfg, "requests", n, "slow", int(st[17]), f"({int(st[17]) / n:.1%})")
