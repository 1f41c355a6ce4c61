#!/bin/bash
# GPU box: the C4 stress leg's always-run kernels -- kernel-trace stats, then two PMC passes
# (stall split; LDS array cycles and bank conflicts), each its own rocprofv3 run.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r6}
N=${STRESS_N:-2000000}
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/alw_${TAG}_kt" -o run --output-format csv \
    -- python3 "$R/scripts/stress_only.py" $N 3 > "$R/gpurun_out/alw_${TAG}_kt.log" 2>&1 || exit $?
if [ -n "$KT_ONLY" ]; then
  cd "$R"; python3 scripts/kstats.py $(find gpurun_out/alw_${TAG}_kt -name "*kernel_stats.csv" | head -1) > gpurun_out/alw_${TAG}_kstats.txt
  head -12 gpurun_out/alw_${TAG}_kstats.txt; grep -h '^{' gpurun_out/alw_${TAG}_kt.log | cut -c1-200; exit 0
fi
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES \
    --kernel-include-regex 'k_waf_always_multi|k_waf_scan|k_waf_direct|k_waf_exact|k_waf_ctx' -d "$R/gpurun_out/alw_${TAG}_sq" -o run --output-format csv \
    -- python3 "$R/scripts/stress_only.py" $N 2 > "$R/gpurun_out/alw_${TAG}_sq.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY \
    --kernel-include-regex 'k_waf_always_multi|k_waf_scan|k_waf_direct|k_waf_exact|k_waf_ctx' -d "$R/gpurun_out/alw_${TAG}_lds" -o run --output-format csv \
    -- python3 "$R/scripts/stress_only.py" $N 2 > "$R/gpurun_out/alw_${TAG}_lds.log" 2>&1 || exit $?
cd "$R"
python3 scripts/kstats.py $(find gpurun_out/alw_${TAG}_kt -name "*kernel_stats.csv" | head -1) > gpurun_out/alw_${TAG}_kstats.txt
head -16 gpurun_out/alw_${TAG}_kstats.txt
grep -h '^{' gpurun_out/alw_${TAG}_kt.log | cut -c1-300
echo done
