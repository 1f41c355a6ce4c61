cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
for d in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --no-cpu --stress-requests 0 --inflight $d --steps 20 > gpurun_out/infl_${d}_$r.log 2>&1 || exit 1
  python3 -c "
import json,sys
l=[x for x in open('gpurun_out/infl_${d}_$r.log') if x.startswith('{')][-1]; d=json.loads(l)
print('inflight ${d} round $r: step %.3f ms scan %.3f route %.3f verify %.3f frac %.3f' % (d['ms_per_step'], d['stage_ms']['scan'], d['stage_ms']['route'], d['stage_ms']['verify'], d['roofline']['frac']))"
done
done
