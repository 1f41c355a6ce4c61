"""Build the committed profile record of the C4 scan that bench.py pairs with its live numbers
(VERDICT r2 "Next round" 1): the rocprofv3 kernel-stats average of k_waf_scan and the PMC
summary (HBM read bytes, LDS bank-conflict rate), stamped with the hash of the kernel sources
they were profiled from.

    python scripts/scan_profile.py TAG KERNEL_STATS_CSV [PMC_SUMMARY_JSON] > profiles/TAG_scan_profile.json

bench.py (roofline) reports `traffic` and `frac_profiled` from this file only when its
`csrc_hash` equals the hash of the tree being benched; otherwise both are null with a reason.
"""
import csv
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ingress-plus_amd", "csrc")
SRC_EXT = (".hip", ".inc", ".cpp", ".hpp", ".h")


def csrc_hash(root: str = ROOT) -> str:
    """sha256 over the kernel and compiler sources (ingress-plus_amd/csrc/*, include/gpumatch.h),
    file names included, in sorted order -- the inputs libgpumatch.so is built from."""
    h = hashlib.sha256()
    csrc = os.path.join(root, "ingress-plus_amd", "csrc")
    files = sorted(f for f in os.listdir(csrc) if f.endswith(SRC_EXT) or f == "Makefile")
    paths = [os.path.join(csrc, f) for f in files] + [os.path.join(root, "include", "gpumatch.h")]
    for p in paths:
        h.update(os.path.relpath(p, root).encode() + b"\0")
        with open(p, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def scan_stats(path: str) -> dict:
    for r in csv.DictReader(open(path)):
        if "k_waf_scan" in r["Name"]:
            return {"k_waf_scan_avg_ns": float(r["AverageNs"]), "k_waf_scan_calls": int(r["Calls"]),
                    "k_waf_scan_min_ns": float(r["MinNs"]), "k_waf_scan_max_ns": float(r["MaxNs"])}
    raise SystemExit(f"no k_waf_scan row in {path}")


def main():
    if sys.argv[1:] == ["--hash"]:   # the Makefile's stamp (gm_buildid.cpp)
        print(csrc_hash())
        return
    tag, stats = sys.argv[1], sys.argv[2]
    rec = {"tag": tag, "csrc_hash": csrc_hash(), "kernel_stats": os.path.basename(stats)}
    rec.update(scan_stats(stats))
    if len(sys.argv) > 3 and os.path.exists(sys.argv[3]):
        s = json.load(open(sys.argv[3]))
        rec["pmc_summary"] = os.path.basename(sys.argv[3])
        rec["pmc_csrc_hash"] = s.get("csrc_hash")
        for k in ("k_waf_scan_hbm_read_bytes_per_launch", "k_waf_scan_lds_bank_conflict_rate"):
            if s.get(k) is not None:
                rec[k] = s[k]
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
