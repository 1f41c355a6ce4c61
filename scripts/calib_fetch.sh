#!/bin/bash
# GPU box: FETCH_SIZE of k_waf_scan for the shipped library and an experiment build ($EXP, e.g.
# exp/cpol0 = GM_SCAN_CPOL=0), same C4 bench run: is the counter's byte count load-policy dependent?
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex 'k_waf_scan' -d $R/gpurun_out/calib_base -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu --stress-requests 0 > $R/gpurun_out/calib_base.log 2>&1 || exit $?
for v in $EXP; do
  GM_LIB=$R/exp/$v/libgpumatch.so timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex 'k_waf_scan' -d $R/gpurun_out/calib_$v -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu --stress-requests 0 > $R/gpurun_out/calib_$v.log 2>&1 || exit $?
  GM_LIB=$R/exp/$v/libgpumatch.so timeout -k 10 300 python -u $R/bench.py --no-cpu --stress-requests 0 > $R/gpurun_out/calib_bench_$v.log 2>&1 || exit $?
done
exit 0
