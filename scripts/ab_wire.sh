#!/bin/bash
# GPU box: the wire-parser bench (bench_next.py --what wire) once per library variant ("main" =
# the in-tree build, NAME = exp/NAME/libgpumatch.so), interleaved ROUNDS times.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-abw}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-main}; do
    if [ "$v" = main ]; then lib=""; else lib="$GRAFT_REPO_ROOT/exp/$v/libgpumatch.so"; fi
    GM_LIB=$lib timeout -k 10 300 python -u scripts/bench_next.py --what wire --cpu-sample 0 > gpurun_out/abw_${TAG}_${v}_$r.log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { tail -5 gpurun_out/abw_${TAG}_${v}_$r.log; exit $rc; }
    python3 - "$v" "gpurun_out/abw_${TAG}_${v}_$r.log" <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[1]:>8s} wire {d['ms_per_call']:.2f} ms/call  {d['value'] / 1e6:.1f} M req/s", flush=True)
PY
  done
done
