#!/bin/bash
# GPU box: the round's closing evidence -- smoke(), the parity suite, the default bench line,
# rocprofv3 kernel stats + PMC passes of the bench, and the secondary config benches.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r1f}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { tail -5 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { tail -20 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_tests_${TAG}.log
TAG=$TAG bash scripts/r1_profile.sh || exit 1
timeout -k 10 600 python scripts/bench_config.py --config c1,c2,c3,c5 > gpurun_out/bench_configs_${TAG}.log 2>&1 || exit 1
grep metric gpurun_out/bench_configs_${TAG}.log | cut -c1-120
