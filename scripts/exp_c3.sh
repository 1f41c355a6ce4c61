#!/bin/bash
# C3 route timing per experiment library (exp/*/libgpumatch.so, scripts/build_exp.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  echo "=== $v"
  GM_LIB=$PWD/exp/$v/libgpumatch.so timeout -k 10 300 python -u scripts/bench_config.py --config ${CFG:-c3} --no-cpu --steps 5 --warmup 1 > gpurun_out/exp_$v.log 2>&1
  rc=$?
  tail -1 gpurun_out/exp_$v.log
  [ $rc -eq 0 ] || exit $rc
done
