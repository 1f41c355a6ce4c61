#!/bin/bash
# GPU box: per-dispatch PMC of C2's route kernels (FAST and SLOW passes), two passes, kernel trace only
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
run() {
  local name=$1; shift
  cd /tmp && TMPDIR=/tmp timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex "k_route" \
    -d "$R/gpurun_out/pmc2_${name}" -o run --output-format csv \
    -- python3 $R/scripts/bench_config.py --config c2 --no-cpu --steps 1 --warmup 0 > "$R/gpurun_out/pmc2_${name}.log" 2>&1
  local rc=$?; cd "$R"; echo "pass $name rc=$rc"; return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU &&
run mem SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS &&
run fetch FETCH_SIZE
