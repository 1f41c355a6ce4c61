#!/bin/bash
# GPU box: the default bench, then the same with the route alone before the scan (stage times alone)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 300 python -u bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/bench_${TAG}.log 2>&1 || exit $?
grep -E "ms route" gpurun_out/bench_${TAG}.log
python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_${TAG}.log').read().strip().splitlines()[-1]); print('overlap: ms/step %.3f value %.3e frac %.3f' % (d['ms_per_step'], d['value'], d['roofline']['frac']))"
timeout -k 10 300 python -u bench.py --no-cpu --serial ${BENCH_ARGS} > gpurun_out/bench_${TAG}_serial.log 2>&1 || exit $?
grep -E "ms route" gpurun_out/bench_${TAG}_serial.log
python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_${TAG}_serial.log').read().strip().splitlines()[-1]); print('serial: ms/step %.3f value %.3e frac %.3f' % (d['ms_per_step'], d['value'], d['roofline']['frac']))"
