#!/bin/bash
# GPU box: the wire parser's parity tests (and the chains through it), then its bench under rocprofv3
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r6w}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "wire or rewrite or consumer or proxy" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_${TAG}.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests_${TAG}.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/scripts/bench_next.py" --what wire --steps 5 --warmup 1 --cpu-sample 2000 > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; tail -2 gpurun_out/prof_${TAG}.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py $(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1) | head -10
