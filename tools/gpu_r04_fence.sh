#!/bin/bash
# Step-program event scope A/B (FBN_PLAN_EVENT_SCOPE): program bit-identity tests with the default,
# then the C3 and C2 program lines per scope, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04fence; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_program.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rnd in 1 2; do
  for sc in system device release_device; do
    FBN_PLAN_EVENT_SCOPE=$sc timeout -k 10 300 python bench.py --mode program --no-cpu-baseline --no-cpu-plan --no-inference \
      --no-fp32 > $O/c3_${sc}_$rnd.json 2> $O/c3_${sc}_$rnd.err || { tail -20 $O/c3_${sc}_$rnd.err; exit 1; }
    echo "c3 $sc $rnd $(grep -o '"ms_per_step": [0-9.]*' $O/c3_${sc}_$rnd.json | head -1)"
  done
done
for sc in system device; do
  FBN_PLAN_EVENT_SCOPE=$sc timeout -k 10 300 python bench.py --mode program --dim 16 --batch 4096 --rows-per-gpu 1000000 \
    --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 > $O/c2_$sc.json 2> $O/c2_$sc.err || { tail -20 $O/c2_$sc.err; exit 1; }
  echo "c2 $sc $(grep -o '"ms_per_step": [0-9.]*' $O/c2_$sc.json | head -1)"
done
