#!/bin/bash
# GPU box script: parity tests, then the default bench, then a rocprofv3 kernel-trace of a short bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r1}
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests.log
tail -25 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest rc=$rc"; exit $rc; fi
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.log 2>&1
rc=$?
tail -6 gpurun_out/bench_${TAG}.log
if [ $rc -ne 0 ]; then echo "stopping: bench rc=$rc"; exit $rc; fi
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log" 2>&1
  rc=$?
  tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log"
  find "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -name "*stats*" | head
fi
exit $rc
