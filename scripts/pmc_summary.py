"""Summarise the rocprofv3 PMC passes written by scripts/pmc.sh into one JSON per round:
per kernel, the mean of every counter over its dispatches, plus the HBM read bytes per launch of
k_waf_scan with the gfx950 FETCH_SIZE correction (x2, MI355X_MICROARCH.md "HBM")."""
import collections
import csv
import json
import os
import sys

out_dir, tag = sys.argv[1], sys.argv[2]
res = collections.defaultdict(dict)
for p in ("fetch", "write", "sq", "lds"):
    f = os.path.join(out_dir, f"pmc_{tag}_{p}", "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        for c, v in d.items():
            res[k][c] = sum(v) / len(v)
            res[k]["dispatches"] = len(v)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from scan_profile import csrc_hash  # noqa: E402
summary = {"tag": tag, "csrc_hash": csrc_hash(), "kernels": res}
scan = res.get("k_waf_scan", {})
if "FETCH_SIZE" in scan:
    summary["k_waf_scan_hbm_read_bytes_per_launch"] = 2.0 * scan["FETCH_SIZE"] * 1024
if "SQ_LDS_BANK_CONFLICT" in scan and scan.get("SQ_LDS_IDX_ACTIVE"):
    # extra LDS cycles from bank conflicts per LDS-active cycle (the scan's Bloom probes)
    summary["k_waf_scan_lds_bank_conflict_rate"] = scan["SQ_LDS_BANK_CONFLICT"] / scan["SQ_LDS_IDX_ACTIVE"]
json.dump(summary, open(os.path.join(out_dir, f"pmc_{tag}_summary.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in summary.items() if k != "kernels"}))
