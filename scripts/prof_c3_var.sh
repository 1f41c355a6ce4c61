#!/bin/bash
# GPU box: rocprofv3 kernel stats of C3 (bench_config.py --config c3) per library variant
# (exp/NAME/libgpumatch.so, scripts/build_exp.sh); summaries in gpurun_out/${TAG}_c3_${v}_kstats.txt
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-pv}
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-main}; do
  d="$R/gpurun_out/prof_${TAG}_c3_$v"
  GM_LIB="$R/exp/$v/libgpumatch.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv \
    -- python3 "$R/scripts/bench_config.py" --config c3 --no-cpu --steps 3 --warmup 1 > "$d.log" 2>&1 || { echo "prof $v failed"; tail -5 "$d.log"; exit 1; }
  f=$(find "$d" -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && python3 "$R/scripts/kstats.py" "$f" > "$R/gpurun_out/${TAG}_c3_${v}_kstats.txt"
  echo "=== $v"; head -8 "$R/gpurun_out/${TAG}_c3_${v}_kstats.txt"
done
exit 0
