#!/bin/bash
# GPU box: rocprofv3 kernel stats of the secondary paths -- C3 (bench_config.py --config c3) and
# the wire parser (bench_next.py --what wire) -- each step under its own time limit.
# Output: gpurun_out/prof_${TAG}_c3/, gpurun_out/prof_${TAG}_wire/ (+ .log), kstats summaries.
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r3}
cd /tmp && export TMPDIR=/tmp
for what in ${WHAT:-c3 wire}; do
  if [ "$what" = wire ]; then
    cmd="$R/scripts/bench_next.py --what wire --steps 3 --warmup 1 --cpu-sample 0"
  else
    cmd="$R/scripts/bench_config.py --config $what --no-cpu --steps 3 --warmup 1"
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_$what" -o run --output-format csv \
    -- python3 $cmd > "$R/gpurun_out/prof_${TAG}_$what.log" 2>&1 || { echo "prof $what failed"; tail -5 "$R/gpurun_out/prof_${TAG}_$what.log"; exit 1; }
  f=$(find "$R/gpurun_out/prof_${TAG}_$what" -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$R/gpurun_out/${TAG}_${what}_kernel_stats.csv" && python3 "$R/scripts/kstats.py" "$f" > "$R/gpurun_out/${TAG}_${what}_kstats.txt"
  cat "$R/gpurun_out/${TAG}_${what}_kstats.txt" | head -14
done
exit 0
