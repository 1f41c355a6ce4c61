#!/bin/bash
# Run bench.py once per "ENV=... --args" variant string; stop at the first failure.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  echo "=== variant $i: $v"
  env $v > /dev/null 2>&1 || true
  timeout -k 10 600 bash -c "$v python bench.py --no-cpu" > gpurun_out/variant_$i.log 2>&1
  rc=$?
  grep -E "steps in|^\{" gpurun_out/variant_$i.log | cut -c1-400
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/variant_$i.log; echo "stopping rc=$rc"; exit $rc; fi
done
