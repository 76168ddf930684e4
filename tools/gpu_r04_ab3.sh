#!/bin/bash
# split-bf16 x3 with 32-deep K tiles (bf16_fwd line, FBN_SPLIT_BWD=1 vs 0) and the C2 stream placement
# under step programs (side passes on the side stream, fold on main; with / without the prefetch).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04ab3; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_kernels.py::test_gemm_split_bf16x3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sp in 1 0; do
  FBN_SPLIT_BWD=$sp timeout -k 10 300 python bench.py --dtype bf16_fwd --no-fp32 --no-cpu-baseline --no-cpu-plan \
    --no-inference --mode program > $O/bf16fwd_split$sp.json 2> $O/bf16fwd_split$sp.err || { tail -20 $O/bf16fwd_split$sp.err; exit 1; }
  echo "split=$sp $(grep -o '"ms_per_step": [0-9.]*' $O/bf16fwd_split$sp.json | head -1)"
done
run() {
  env $2 timeout -k 10 200 python bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 \
    --no-inference --no-cpu-plan --mode program $3 > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.json | head -1)"
}
run c2_base "FBN_X=0" "" && run c2_side_nofix "FBN_SIDE_SERIAL=0 FBN_FIXUP_ON_SIDE=0" "" \
  && run c2_side_nofix_nopf "FBN_SIDE_SERIAL=0 FBN_FIXUP_ON_SIDE=0" "--no-prefetch" && run c2_nopf "FBN_X=0" "--no-prefetch" \
  && run c2_side_nofix2 "FBN_SIDE_SERIAL=0 FBN_FIXUP_ON_SIDE=0" "" && run c2_base2 "FBN_X=0" ""
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python $R/bench.py --dtype bf16_fwd --no-fp32 --no-cpu-baseline --no-cpu-plan --no-inference --steps 20 --mode program \
  > $O/prof.log 2>&1 || exit 1
