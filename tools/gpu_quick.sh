#!/bin/bash
# Quick GPU-box iteration: a pytest selection (-k expression) then the bench without the CPU baseline.
# Usage (via gpurun): bash tools/gpu_quick.sh <tag> "<pytest -k expr>" [bench args...]
set -o pipefail
TAG=$1; K=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest $R/tests -q -m gpu -k "$K" -p no:cacheprovider --timeout 180 --timeout-method thread \
    > $OUT/tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -4 $OUT/tests_$TAG.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 600 python $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench_$TAG.err
python - "$OUT/bench_$TAG.json" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    print("ms/step", d["ms_per_step"], "value", d["value"], "fp32", d.get("fp32", {}).get("ms_per_step"))
    for r in d["rooflines"]:
        print(f'  {r["kernel"][:60]:60s} {r["avg_launch_ms"]*1e3:8.1f} us  {r["achieved"]:8.1f} {r["unit"]}  frac {r["frac"]}')
PY
exit $rc
