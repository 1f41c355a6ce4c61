#!/bin/bash
# GPU box: the routing configs (C1 / C2 / C3 / C5, scripts/bench_config.py) once per library
# variant ("main" = the in-tree build, else exp/NAME/libgpumatch.so).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-abc}
for c in ${CONFIGS:-c1 c2 c3 c5}; do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=""; else lib="$GRAFT_REPO_ROOT/exp/$v/libgpumatch.so"; fi
    GM_LIB=$lib timeout -k 10 300 python -u scripts/bench_config.py --config $c --no-cpu --steps 5 --warmup 1 > gpurun_out/abc_${TAG}_${c}_${v}.log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { tail -5 gpurun_out/abc_${TAG}_${c}_${v}.log; exit $rc; }
    python3 - "$c" "$v" "gpurun_out/abc_${TAG}_${c}_${v}.log" <<'PY'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[1]} {sys.argv[2]:>8s} {d.get('ms_per_step', 0):8.3f} ms  {d.get('value', 0) / 1e6:9.1f} M/s", flush=True)
PY
  done
done
