#!/bin/bash
# Binned table-Adam prefetch: bit-identity tests, then the C3 bench with the binned prefetch and with
# adam_prefetch2 (FBN_PF_BINNED=0), short lines (no embedded fp32 / inference / CPU legs); the
# launcher's training-run AUC parity; then the kernel-trace profiles (headline + one-rank sharded).
set -o pipefail
OUT=gpurun_out/${1:-r04pf}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
    "tests/test_gpu_trainer.py::test_next_batch_prefetch_bit_identical" tests/test_gpu_program.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for arm in 1 0 1 e; do
  if [ $arm = e ]; then ENV="FBN_WGRAD_EARLY=1"; else ENV="FBN_PF_BINNED=$arm"; fi
  env $ENV timeout -k 10 300 python -u bench.py --no-fp32 --no-inference --no-cpu-baseline > $OUT/bench_pf$arm.json 2> $OUT/bench_pf$arm.err
  rc=$?; echo "bench $ENV rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_pf$arm.json)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread \
    "tests/test_launcher.py::test_launcher_auc_parity_vs_reference_loop" > $OUT/launcher.log 2>&1
rc=$?; echo "launcher rc=$rc"; [ $rc -le 1 ] || exit $rc
bash tools/gpu_prof.sh r04pf --no-fp32 --no-inference --no-cpu-plan > /dev/null || exit $?
bash tools/shard_prof.sh r04pf_shard || exit $?
