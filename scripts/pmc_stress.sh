#!/bin/bash
# GPU box: PMC passes over the C4 stress leg (scripts/stress_only.py), WAF kernels only; one counter
# group per rocprofv3 run.  Output: gpurun_out/pmcs_${TAG}_<pass>/.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-s}
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex 'k_waf' \
    -d "$GRAFT_REPO_ROOT/gpurun_out/pmcs_${TAG}_${name}" -o run --output-format csv \
    -- python "$GRAFT_REPO_ROOT/scripts/stress_only.py" ${N:-500000} 1 > "$GRAFT_REPO_ROOT/gpurun_out/pmcs_${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "pmc pass $name rc=$rc"
  return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU &&
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
