#!/bin/bash
# tools/ab_arms2.sh with extra bench.py arguments shared by every arm (e.g. the C2 shape).
# Usage (via gpurun): bash tools/ab_arms3.sh <rounds> "<bench args>" "VAR=a" "VAR=b VAR2=c" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
ARGS=$1; shift
mkdir -p $R/gpurun_out
for i in $(seq 1 $N); do
  for e in "$@"; do
    (export FBN_AB_ARM=1 $e; timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-fp32 --no-inference $ARGS \
       > $R/gpurun_out/abarm.json 2>/dev/null) || exit 1
    echo "arm [$e] round $i $(python -c "
import json; d=json.loads(open('$R/gpurun_out/abarm.json').read().splitlines()[-1])
print(d['ms_per_step'], 'gather', d['rooflines'][0]['frac'], 'top', d['roofline']['kernel'][:24], d['roofline']['frac'])")"
  done
done
