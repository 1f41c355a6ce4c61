#!/bin/bash
# GPU box: the C4 stress leg alone (scripts/stress_only.py) once per library variant ("main" = the
# in-tree build, NAME = exp/NAME/libgpumatch.so), interleaved ROUNDS times.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-sab}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=""; else lib="$GRAFT_REPO_ROOT/exp/$v/libgpumatch.so"; fi
    GM_LIB=$lib timeout -k 10 200 python scripts/stress_only.py ${STRESS_N:-2000000} 5 > gpurun_out/stress_${TAG}_${v}_$r.log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { tail -5 gpurun_out/stress_${TAG}_${v}_$r.log; exit $rc; }
    python3 - "$v" "gpurun_out/stress_${TAG}_${v}_$r.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
s = d["stage_ms"]
print(f"{sys.argv[1]:>8s} step {d['ms_per_step']:.2f} ms  route {s['route']:.2f} scan {s['scan']:.2f} verify {s['verify']:.2f} "
      f"tail {s['tail']:.2f}", flush=True)
PY
  done
done
