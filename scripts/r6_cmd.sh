cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/pmc_c3.sh && bash scripts/pmc_c2.sh && python3 scripts/pmc_read.py gpurun_out/pmc3 > gpurun_out/pmc3_r6fin.txt && python3 scripts/pmc_read.py gpurun_out/pmc2 > gpurun_out/pmc2_r6fin.txt; wc -l gpurun_out/pmc3_r6fin.txt gpurun_out/pmc2_r6fin.txt
