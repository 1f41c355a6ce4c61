#!/bin/bash
# GPU box: parity tests, then the bench at several scan prefetch depths (GM_SCAN_DEPTH).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/bench_variants.sh ${VARIANTS:-"GM_SCAN_DEPTH=1" "GM_SCAN_DEPTH=2" "GM_SCAN_DEPTH=4" "GM_SCAN_DEPTH=6"}
