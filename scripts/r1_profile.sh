#!/bin/bash
# GPU box: the round's evidence -- bench line, rocprofv3 kernel stats, PMC passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r1b}
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.log 2>&1 || { tail -5 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log | cut -c1-300
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log" 2>&1 ) || { echo "rocprof stats failed"; exit 1; }
f=$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/${TAG}_kernel_stats.csv && python3 scripts/kstats.py "$f" | head -8
TAG=$TAG bash scripts/pmc.sh
