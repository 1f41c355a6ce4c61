#!/bin/bash
# GPU box: PMC passes (instruction mix / waits; LDS; FETCH_SIZE) of the route-stage kernels on the
# routing configs C1/C2/C3/C5 (scripts/bench_config.py, 2M requests, 1 step).  Output:
# gpurun_out/pmcc_<cfg>_<pass>/ (scripts/pmc_read.py summarises them).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in ${CFGS:-c1 c2 c3 c5}; do
  TAG=$c KRE='k_route|k_rloc' PMC_CMD="scripts/bench_config.py --config $c --no-cpu --steps 1 --warmup 0 --requests 2000000 --pool 1000000" \
    bash scripts/pmc_cmd.sh || exit $?
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex 'k_route|k_rloc' \
    -d "$GRAFT_REPO_ROOT/gpurun_out/pmcc_${c}_fetch" -o run --output-format csv \
    -- python "$GRAFT_REPO_ROOT/scripts/bench_config.py" --config $c --no-cpu --steps 1 --warmup 0 --requests 2000000 --pool 1000000 \
    > "$GRAFT_REPO_ROOT/gpurun_out/pmcc_${c}_fetch.log" 2>&1 || exit $?
  echo "pmc pass fetch rc=0"
  cd "$GRAFT_REPO_ROOT"
done
exit 0
