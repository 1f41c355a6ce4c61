#!/bin/bash
# round-3 scan / route A/B batch (variants under exp/, see scripts/build_exp.sh)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && ROUNDS=${ROUNDS:-2} TAG=${TAG:-s2} bash scripts/ab.sh ${VARIANTS:-main norec s4 noblk nohost bpc3 bpc1}
