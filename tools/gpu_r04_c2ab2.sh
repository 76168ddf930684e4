#!/bin/bash
# C2 under step programs after the d < 128 weight gradients joined the grouped slab launch: the line,
# without the next-batch prefetch, with lazy windows 16 / 64 (default 32), and the side-stream variant.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c2ab2; mkdir -p $O
cd $R
run() {
  env $2 timeout -k 10 200 python bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 \
    --no-inference --no-cpu-plan --mode program $3 > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.json | head -1)"
}
run base "FBN_X=0" "" && run nopf "FBN_X=0" "--no-prefetch" && run w16 "FBN_X=0" "--lazy-window 16" \
  && run w64 "FBN_X=0" "--lazy-window 64" && run side_nofix "FBN_SIDE_SERIAL=0 FBN_FIXUP_ON_SIDE=0" "" \
  && run base2 "FBN_X=0" ""
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python $R/bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 --no-inference \
  --no-cpu-plan --mode program --steps 20 > $O/prof.log 2>&1 || exit 1
