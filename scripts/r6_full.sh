#!/bin/bash
# GPU box: the whole GPU suite, the C4 bench, the wire bench under rocprofv3 (one call)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r6}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_${TAG}.log 2>&1
rc=$?; echo "pytest exit=$rc" >> gpurun_out/gpu_tests_${TAG}.log; tail -4 gpurun_out/gpu_tests_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/bench_${TAG}.log 2>&1
rc=$?; grep -h "steps in\|stress\]" gpurun_out/bench_${TAG}.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_wire" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/scripts/bench_next.py" --what wire --steps 5 --warmup 1 --cpu-sample 2000 > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_wire.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; [ $rc -eq 0 ] || { tail -3 gpurun_out/prof_${TAG}_wire.log; exit $rc; }
grep -h "wire" gpurun_out/prof_${TAG}_wire.log | tail -2 | cut -c1-400
python3 scripts/kstats.py $(find gpurun_out/prof_${TAG}_wire -name "*kernel_stats.csv" | head -1) | head -8
