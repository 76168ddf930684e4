#!/bin/bash
# Kernel trace + stats of the headline bench (step programs) and of C2, the per-step timelines of the
# timed replays, traces gzipped (gpurun copies back <= 64 MiB).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04tr; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- \
  python $R/bench.py --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 --prime 64 --steps 20 --warmup 5 \
  > $O/c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- \
  python $R/bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-cpu-plan --no-inference \
  --no-fp32 --prime 64 --steps 20 --warmup 5 > $O/c2.log 2>&1 || exit 1
cd $R
for c in c3 c2; do
  gzip -f $O/$c/run_kernel_trace.csv
done
ls -la $O/c3 $O/c2
