"""bench.py's C4 stress leg alone (for profiling): python scripts/stress_only.py [requests] [steps]"""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd"))
import json  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
from gpumatch import engine, records, workloads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
args = types.SimpleNamespace(stress_requests=n, steps=steps, warmup=1)
print(json.dumps(bench.stress_leg(torch, engine, records, workloads, args, 0)))
