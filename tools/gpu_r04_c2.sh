#!/bin/bash
# C2 (d 16, 1 M rows, B 4096): the bench line (launch-mode trial incl. step programs) and a kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c2; mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 \
  --no-inference --no-cpu-plan > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
tail -1 $O/c2.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python $R/bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 --no-inference \
  --no-cpu-plan --steps 20 > $O/prof.log 2>&1 || exit 1
