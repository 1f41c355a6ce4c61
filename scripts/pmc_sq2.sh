#!/bin/bash
# GPU box: the stall split of the C4 scan / context / exact kernels (SQ_WAIT_INST_ANY and
# SQ_WAIT_INST_LDS beside the active-instruction counters), one rocprofv3 --pmc pass, kernel trace only.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r6}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VALU \
    --kernel-include-regex 'k_waf_(scan|ctx|exact)' -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_sq2" -o run --output-format csv \
    -- python "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu --no-alone --stress-requests 0 ${BENCH_ARGS} \
    > "$GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_sq2.log" 2>&1
rc=$?
echo "pmc sq2 rc=$rc"
exit $rc
