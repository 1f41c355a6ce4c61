#!/bin/bash
# GPU box: bench variants (env strings as args), then a kernel trace of a short bench under $PROF_ENV.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-rx}
bash scripts/bench_variants.sh "$@" || exit $?
cd /tmp && export TMPDIR=/tmp
for m in ${PROF_MODES:-1}; do
  GM_ROUTE_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_m$m" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_m$m.log" 2>&1 || { echo "rocprof failed"; exit 1; }
  f=$(find "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_m$m" -name "*kernel_stats.csv" | head -1)
  python3 "$GRAFT_REPO_ROOT/scripts/kstats.py" "$f" | head -8
done
