#!/bin/bash
# Split-bf16 x3 backward GEMMs of the bf16_fwd mode and the d < 128 fused bilinear / grouped weight
# gradients: kernel tests, the precision-mode parity tests, the program bit-identity tests, then the
# bf16_fwd bench line with split (default) and fp32 MFMA, and the C2 A/B lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04split; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  "tests/test_gpu_kernels.py::test_gemm_split_bf16x3" "tests/test_gpu_kernels.py::test_fused_bilinear_matches_unfused_math" \
  "tests/test_gpu_program.py" "tests/test_gpu_coverage.py::test_auc_precision_modes_vs_oracle" \
  "tests/test_gpu_coverage.py::test_config_size_trainer_step" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for sp in 1 0; do
  FBN_SPLIT_BWD=$sp timeout -k 10 300 python bench.py --dtype bf16_fwd --no-fp32 --no-cpu-baseline --no-cpu-plan \
    --no-inference > $O/bench_split$sp.json 2> $O/bench_split$sp.err || { tail -20 $O/bench_split$sp.err; exit 1; }
  echo "split=$sp $(grep -o '"ms_per_step": [0-9.]*' $O/bench_split$sp.json | head -1)"
done
bash tools/gpu_r04_c2ab2.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python $R/bench.py --dtype bf16_fwd --no-fp32 --no-cpu-baseline --no-cpu-plan --no-inference --steps 20 \
  > $O/prof.log 2>&1 || exit 1
