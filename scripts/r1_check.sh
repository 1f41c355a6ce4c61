#!/bin/bash
# GPU box: parity tests, full-pool parity against the oracle, then the bench (variants optional).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
if [ -z "$NO_POOL" ]; then
  timeout -k 10 400 python -u scripts/pool_parity.py > gpurun_out/pool_parity.log 2>&1
  rc=$?
  head -4 gpurun_out/pool_parity.log
  [ $rc -eq 0 ] || { tail -30 gpurun_out/pool_parity.log; exit $rc; }
fi
bash scripts/bench_variants.sh ${VARIANTS:-"GM_SCAN_DEPTH=4"}
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  rc=$?
  f=$(find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && python3 "$GRAFT_REPO_ROOT/scripts/kstats.py" "$f" | head -14
  exit $rc
fi
