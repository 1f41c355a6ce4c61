#!/bin/bash
# GPU box: the round's measurement set on one tree, after scripts/gpu_round.sh (tests, bench, kernel
# stats, PMC): the routing configs with their route-kernel time, C3 and C4-stress kernel stats,
# the wire parser and peer-selection benches, smoke().  Every GPU step has its own time limit;
# the first failure ends the call.  Output: gpurun_out/${TAG}_*.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r5e}
step() {   # name, limit (s), command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_${name}.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/${TAG}_${name}.txt"
  return $rc
}
step configs 400 bash -c 'for c in c1 c2 c3 c5; do python -u scripts/bench_config.py --config $c --no-cpu || exit 1; done' &&
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
step next 400 python -u scripts/bench_next.py --what peers,peers-default,wire --cpu-sample 2000 &&
cd /tmp && export TMPDIR=/tmp &&
step c3prof 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_c3" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/scripts/bench_config.py" --config c3 --no-cpu --steps 3 --warmup 1 &&
step stressprof 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_stress" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/scripts/stress_only.py" 2000000 3 &&
cd "$GRAFT_REPO_ROOT" &&
for k in c3 stress; do
  f=$(find gpurun_out/prof_${TAG}_$k -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" gpurun_out/${TAG}_${k}_kernel_stats.csv
done
exit $?
