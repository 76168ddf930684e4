#!/bin/bash
# Interleaved A/B/... of environment settings over the default bf16 bench (no CPU baseline, no
# fp32 line).  Usage (via gpurun): bash tools/ab_arms.sh <rounds> "VAR=a" "VAR=b VAR2=c" ...
# An empty arm ("") is the default; BENCH_ARGS="..." in an arm adds bench arguments.
# Prints ms/step per arm and round.
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
mkdir -p $R/gpurun_out
for i in $(seq 1 $N); do
  for e in "$@"; do
    (export BENCH_ARGS= $e; timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-fp32 $BENCH_ARGS \
       > $R/gpurun_out/abarm.json 2>/dev/null) || exit 1
    echo "arm [$e] round $i $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/abarm.json)"
  done
done
