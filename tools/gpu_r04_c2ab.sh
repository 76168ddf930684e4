#!/bin/bash
# C2 launch-structure A/B under step programs: side passes in sequence on the main stream (default at
# d < 128) vs on the side stream, with and without the claims on the side stream.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c2ab; mkdir -p $O
cd $R
run() {
  env $2 timeout -k 10 200 python bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 \
    --no-inference --no-cpu-plan --mode program > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.json | head -1)"
}
run base "FBN_SIDE_SERIAL=auto" && run side "FBN_SIDE_SERIAL=0" && run side_claim "FBN_SIDE_SERIAL=0 FBN_CLAIM_ON_SIDE=1" \
  && run side_nofix "FBN_SIDE_SERIAL=0 FBN_FIXUP_ON_SIDE=0" && run base2 "FBN_SIDE_SERIAL=auto"
