# the final tree: the gather tests, then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_coverage.py tests/test_gpu_trainer.py > gpurun_out/s2t_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/s2t_bench.json 2> gpurun_out/s2t_bench.err
