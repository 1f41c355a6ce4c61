#!/bin/bash
# GPU box: kernel stats of the C4 pipeline at several batch / pool sizes (does the exact check's
# time per survivor depend on the arena's footprint?)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for cfg in "1000000 1000000" "10000000 1000000" "10000000 100000"; do
  set -- $cfg
  d="$GRAFT_REPO_ROOT/gpurun_out/sz_$1_$2"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu --no-alone --stress-requests 0 --requests $1 --pool $2 > "$d.log" 2>&1 || { tail -5 "$d.log"; exit 1; }
  f=$(find "$d" -name "*kernel_stats.csv" | head -1)
  echo "== requests $1 pool $2"; grep "status words\|candidates" "$d.log"
  python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if any(k in x['Name'] for k in ('k_waf_exact', 'k_waf_ctx', 'k_waf_scan', 'k_route')):
        print(f"{x['Name'][:40]:40s} {float(x['AverageNs'])/1e3:9.1f} us")
PY
done
