#!/bin/bash
# GPU box, round 6 final tree, part B: smoke, the routing configs, the wire bench, the stress leg's kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r6end}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_${TAG}.log 2>&1 || { tail -5 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
# the default bench again, now that profiles/ holds this tree's scan profile (frac_profiled, traffic)
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench2_${TAG}.log 2>&1 || { tail -5 gpurun_out/bench2_${TAG}.log; exit 1; }
grep -h '^{' gpurun_out/bench2_${TAG}.log | cut -c1-300
: > gpurun_out/${TAG}_configs.txt
for c in c1 c2 c3 c5; do
  timeout -k 10 300 python3 -u scripts/bench_config.py --config $c --no-cpu --steps 10 --warmup 2 > gpurun_out/cfg_${TAG}_$c.log 2>&1 || { tail -5 gpurun_out/cfg_${TAG}_$c.log; exit 1; }
  grep -h '^{' gpurun_out/cfg_${TAG}_$c.log >> gpurun_out/${TAG}_configs.txt
done
python3 - <<PY
import json
for l in open("gpurun_out/${TAG}_configs.txt"):
    d = json.loads(l); print(d["config"], round(d["ms_per_step"], 3), "ms", round(d["value"] / 1e6, 1), "M/s")
PY
timeout -k 10 300 python3 -u scripts/bench_next.py --what wire --cpu-sample 2000 > gpurun_out/wire_${TAG}.log 2>&1 || exit 1
grep -h '^{' gpurun_out/wire_${TAG}.log | cut -c1-200
timeout -k 10 300 python3 -u scripts/bench_next.py --what peers > gpurun_out/peers_${TAG}.log 2>&1 || exit 1
grep -h '^{' gpurun_out/peers_${TAG}.log | cut -c1-200
KT_ONLY=1 TAG=$TAG bash scripts/pmc_alw.sh || exit 1
if [ -n "$C2PMC" ]; then bash scripts/pmc_c2.sh && python3 scripts/pmc_read.py gpurun_out/pmc2 > gpurun_out/pmc2_${TAG}.txt; fi
