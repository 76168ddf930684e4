#!/bin/bash
# Round 4 GPU evidence run: the new parity tests (step programs, C4 8-rank rehearsal, the benched call
# at C3, multi-rank, the launcher's training-run AUC), then the default bench line.  Each GPU step has
# its own time limit; the bench runs only after a test run that ended normally (rc 0 or 1: passed, or
# assertion failures) -- never after a time limit, an abort or a crash.
set -o pipefail
OUT=gpurun_out/${1:-r04}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v --timeout 800 --timeout-method thread \
    tests/test_gpu_program.py tests/test_gpu_c4.py "tests/test_gpu_coverage.py::test_auc_precision_modes_vs_oracle" \
    tests/test_gpu_multirank.py "tests/test_launcher.py::test_launcher_auc_parity_vs_reference_loop" > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 420 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc2=$?; echo "bench rc=$rc2"; exit $(( rc2 != 0 ? rc2 : rc ))
