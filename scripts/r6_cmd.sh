cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ROUNDS=2 TAG=$TAG bash scripts/stress_ab.sh main clsu8 || exit $?
CONFIGS="c3" TAG=$TAG bash scripts/ab_configs.sh main clsu8
