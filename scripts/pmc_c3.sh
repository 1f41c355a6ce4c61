cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex "k_rloc_multi" \
    -d "$GRAFT_REPO_ROOT/gpurun_out/pmc3_${name}" -o run --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/scripts/bench_config.py --config c3 --no-cpu --steps 1 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/pmc3_${name}.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU &&
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES &&
run fetch FETCH_SIZE
