#!/bin/bash
# GPU box: the WAF parity tests, then bench variants ("ENV=..." strings) -- a quick kernel iteration.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "${TESTS:-waf or c4}" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -4 gpurun_out/quick_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/quick_tests.log | head -20; exit $rc; }
bash scripts/bench_variants.sh "$@"
