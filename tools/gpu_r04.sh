#!/bin/bash
# Round 4 GPU evidence run: new parity tests (C4 8-rank rehearsal, step programs, the benched call at
# C3), then the default bench line.  Each GPU step has its own time limit; steps chained with &&.
set -o pipefail
OUT=gpurun_out/${1:-r04}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread \
    tests/test_gpu_program.py tests/test_gpu_c4.py "tests/test_gpu_coverage.py::test_auc_precision_modes_vs_oracle" \
    tests/test_gpu_multirank.py "tests/test_launcher.py::test_launcher_auc_parity_vs_reference_loop" > $OUT/tests.log 2>&1 &&
timeout -k 10 420 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
