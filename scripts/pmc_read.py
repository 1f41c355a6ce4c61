"""Per-kernel sums of a pmc_cmd.sh run: python scripts/pmc_read.py gpurun_out/pmcc_<tag>"""
import collections
import csv
import glob
import sys

for p in ("sq", "lds", "fetch"):
    fs = glob.glob(f"{sys.argv[1]}_{p}/**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:44]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", ""))
    for k, v in agg.items():
        nd = max(1, len(disp[k]))
        print(p, k, nd, {a: f"{b / nd:.3g}" for a, b in sorted(v.items())})
