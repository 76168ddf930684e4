#!/bin/bash
# One join of the side stream per step (the second, redundant one removed): program / trainer tests and
# two bench lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04join; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_program.py \
  tests/test_gpu_trainer.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 > $O/bench$k.json 2> $O/bench$k.err \
    || { tail -20 $O/bench$k.err; exit 1; }
  echo "bench$k $(grep -o '"ms_per_step": [0-9.]*' $O/bench$k.json | head -1)"
done
