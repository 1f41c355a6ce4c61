#!/bin/bash
# GPU box: rocprofv3 kernel stats of the C4 bench per library variant ("main" = the in-tree build,
# NAME = exp/NAME/libgpumatch.so), the kernels named in KSEL summarised one line per variant.
# Every GPU step has its own time limit; the first failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-pv}
KSEL=${KSEL:-k_waf_exact,k_waf_ctx,k_waf_scan}
for v in "$@"; do
  if [ "$v" = main ]; then export GM_LIB=""; else export GM_LIB="$GRAFT_REPO_ROOT/exp/$v/libgpumatch.so"; fi
  d="$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_$v"
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu --no-alone --stress-requests 0 \
         --allow-nondefault-build ${BENCH_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_$v.log" 2>&1)
  rc=$?
  [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; tail -5 "gpurun_out/prof_${TAG}_$v.log"; exit $rc; }
  f=$(find "$d" -name "*kernel_stats.csv" | head -1)
  python3 - "$v" "$f" "$KSEL" <<'PY'
import csv, sys
v, f, ks = sys.argv[1], sys.argv[2], sys.argv[3].split(",")
rows = {r["Name"]: r for r in csv.DictReader(open(f))}
out = []
for k in ks:
    m = [r for n, r in rows.items() if k + "(" in n or k + "<" in n]
    if m:
        out.append(f"{k} {sum(float(r['AverageNs']) for r in m) / 1e3:.1f} us")
print(f"{v:>6s}: " + "  ".join(out), flush=True)
PY
  grep -h "status words\|exact-check\|steps in" "gpurun_out/prof_${TAG}_$v.log" | sed "s/^/    /"
done
