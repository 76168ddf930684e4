#!/bin/bash
# BN1 backward partials in the dgrad epilogue at C2 (16-row chunks): kernel tests, the C2 / C3 one-step
# parity tests and the C2 program line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c2b; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_program.py "tests/test_gpu_coverage.py::test_config_size_trainer_step" > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  timeout -k 10 300 python bench.py --mode program --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline \
    --no-cpu-plan --no-inference --no-fp32 > $O/c2_$k.json 2> $O/c2_$k.err || { tail -20 $O/c2_$k.err; exit 1; }
  echo "c2 $k $(grep -o '"ms_per_step": [0-9.]*' $O/c2_$k.json | head -1)"
done
