#!/bin/bash
# GPU box: optional parity subset (PYTEST_K), then the C4 bench once per library variant
# ("name" = exp/name/libgpumatch.so, "main" = the in-tree build), interleaved ROUNDS times so that
# box drift hits every variant alike.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "$PYTEST_K" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests_${TAG}.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests_${TAG}.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=""; else lib="$GRAFT_REPO_ROOT/exp/$v/libgpumatch.so"; fi
    GM_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu --stress-requests 0 --allow-nondefault-build ${BENCH_ARGS} > gpurun_out/ab_${TAG}_${v}_$r.log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_${TAG}_${v}_$r.log; exit $rc; }
    python3 - "$v" "gpurun_out/ab_${TAG}_${v}_$r.log" <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line); r = d["roofline"]
print(f"{sys.argv[1]:>8s} step {d['ms_per_step']:.3f} ms  scan {d['stage_ms']['scan']:.3f} route {d['stage_ms']['route']:.3f} "
      f"verify {d['stage_ms']['verify']:.3f} ralone {d['stage_ms'].get('route_alone', 0):.3f}  frac {r['frac']:.3f} alone {r.get('scan_alone_ms', 0):.3f} ({r.get('frac_alone', 0):.3f})", flush=True)
PY
  done
done
