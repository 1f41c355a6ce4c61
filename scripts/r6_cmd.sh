cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cfg_${TAG}_c2 -o run --output-format csv \
   -- python3 $R/scripts/bench_config.py --config c2 --no-cpu --steps 5 --warmup 1 > $R/gpurun_out/cfg_${TAG}_c2.log 2>&1 || exit $?
cd $R && python3 scripts/kstats.py $(find gpurun_out/cfg_${TAG}_c2 -name "*kernel_stats.csv" | head -1) | head -4
