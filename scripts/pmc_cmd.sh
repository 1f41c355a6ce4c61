#!/bin/bash
# GPU box: two PMC passes (instruction mix / waits; LDS) over `python $PMC_CMD`, kernels matching
# $KRE only; one counter group per rocprofv3 run.  Output: gpurun_out/pmcc_${TAG}_<pass>/.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-c}
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex "${KRE:-k_}" \
    -d "$GRAFT_REPO_ROOT/gpurun_out/pmcc_${TAG}_${name}" -o run --output-format csv \
    -- python $GRAFT_REPO_ROOT/$PMC_CMD > "$GRAFT_REPO_ROOT/gpurun_out/pmcc_${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "pmc pass $name rc=$rc"
  return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU &&
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
