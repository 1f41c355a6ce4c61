cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_${TAG}.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_${TAG}.log; [ $rc -eq 0 ] || exit $rc
KT_ONLY=1 bash scripts/pmc_alw.sh || exit $?
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/bench_${TAG}.log 2>&1 || exit $?
grep -h '"metric"' gpurun_out/bench_${TAG}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4', d['ms_per_step'], d['stage_ms'], 'stress', d['stress']['ms_per_step'], d['stress']['stage_ms'])"
