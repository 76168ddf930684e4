#!/bin/bash
# Binned table-Adam prefetch: bit-identity tests, then the C3 bench with the binned prefetch and with
# adam_prefetch2 (FBN_PF_BINNED=0), short lines (no embedded fp32 / inference / CPU legs).
set -o pipefail
OUT=gpurun_out/${1:-r04pf}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
    "tests/test_gpu_trainer.py::test_next_batch_prefetch_bit_identical" tests/test_gpu_program.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for arm in 1 0 1; do
  FBN_PF_BINNED=$arm timeout -k 10 300 python -u bench.py --no-fp32 --no-inference --no-cpu-baseline > $OUT/bench_pf$arm.json 2> $OUT/bench_pf$arm.err
  rc=$?; echo "bench binned=$arm rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_pf$arm.json)"; [ $rc -eq 0 ] || exit $rc
done
