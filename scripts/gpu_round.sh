#!/bin/bash
# GPU box: parity tests (-m gpu), then the default bench; optional rocprofv3 kernel stats (PROF=1)
# and PMC passes (PMC=1).  Every GPU step has its own time limit; the first failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r2}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu ${PYTEST_K:+-k "$PYTEST_K"} --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_${TAG}.log 2>&1
  rc=$?
  echo "pytest exit=$rc" >> gpurun_out/gpu_tests_${TAG}.log
  tail -30 gpurun_out/gpu_tests_${TAG}.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.log 2>&1
  rc=$?
  tail -4 gpurun_out/bench_${TAG}.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu --no-alone --stress-requests 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log" 2>&1
  rc=$?
  tail -2 "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log"
  [ $rc -eq 0 ] || exit $rc
  cd "$GRAFT_REPO_ROOT"
  f=$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" gpurun_out/${TAG}_kernel_stats.csv && python3 scripts/kstats.py "$f" | head -8
fi
if [ -n "$PMC" ]; then
  TAG=$TAG bash scripts/pmc.sh || exit $?
fi
if [ -f gpurun_out/${TAG}_kernel_stats.csv ]; then
  python3 scripts/scan_profile.py $TAG gpurun_out/${TAG}_kernel_stats.csv gpurun_out/pmc_${TAG}_summary.json > gpurun_out/${TAG}_scan_profile.json
fi
exit 0
