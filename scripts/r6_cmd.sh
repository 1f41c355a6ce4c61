cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
CONFIGS="c2" TAG=$TAG bash scripts/ab_configs.sh main slow5 slow6 main slow5 slow6
