#!/bin/bash
# C2 step programs: kernel + HIP runtime trace (which API calls sit between the step's kernels).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c2t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/prof -o run -- \
  python $R/bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 --no-inference \
  --no-cpu-plan --mode program --steps 10 --warmup 5 > $O/prof.log 2>&1 || exit 1
