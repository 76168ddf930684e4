#!/bin/bash
# MLP input rows padded to a multiple of 64 below d = 128 (C2: layer 1 on the LDS-DMA kernel): the
# whole -m gpu suite, then two C2 lines and the C3 line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04pad; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -q -m gpu tests -p no:cacheprovider --timeout 600 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -le 1 ] || exit $rc
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -5
for k in 1 2; do
  timeout -k 10 300 python bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-cpu-plan \
    --no-inference --no-fp32 > $O/c2_$k.json 2> $O/c2_$k.err || { tail -20 $O/c2_$k.err; exit 1; }
  echo "c2 $k $(grep -o '"ms_per_step": [0-9.]*' $O/c2_$k.json | head -1)"
done
timeout -k 10 400 python bench.py --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 > $O/c3.json 2> $O/c3.err \
  || { tail -20 $O/c3.err; exit 1; }
echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $O/c3.json | head -1)"
