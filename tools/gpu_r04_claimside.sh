#!/bin/bash
# Row claims on the side stream under step programs (device-scope edges), interleaved A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04cs; mkdir -p $O
cd $R
for rnd in 1 2; do
  for cs in 0 1; do
    FBN_CLAIM_ON_SIDE=$cs timeout -k 10 300 python bench.py --mode program --no-cpu-baseline --no-cpu-plan --no-inference \
      --no-fp32 --no-live-probes > $O/cs${cs}_$rnd.json 2> $O/cs${cs}_$rnd.err || { tail -20 $O/cs${cs}_$rnd.err; exit 1; }
    echo "claim_on_side=$cs $rnd $(grep -o '"ms_per_step": [0-9.]*' $O/cs${cs}_$rnd.json | head -1)"
  done
done
