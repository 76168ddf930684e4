#!/bin/bash
# A/B of the next-batch prefetch in one GPU call (interleaved runs; DVFS/box noise is ~3 %).
# Usage (via gpurun): bash tools/ab_prefetch.sh [rounds] [extra bench args...]
N=${1:-3}; shift
for i in $(seq $N); do
  for arm in "" "--no-prefetch"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32 $arm "$@" 2>/dev/null | python -c "
import json,sys
d=json.loads(sys.stdin.readline())
print('arm ${arm:-prefetch}', d['ms_per_step'], [(r['kernel'][:14], round(r['avg_launch_ms']*1e3,1)) for r in d['rooflines']])" || exit 1
  done
done
