# remaining round-3 measurements: one-step parity (bf16 modes), full bench line, window A/B, GEMM lab,
# C5 shard test + lines, kernel trace of the C3 bench
set -o pipefail
mkdir -p gpurun_out/parity
FBN_PARITY_OUT=gpurun_out/parity timeout -k 10 300 python -u -m pytest tests/test_gpu_coverage.py -x -v -s --timeout 250 --timeout-method thread -k "trainer_step" > gpurun_out/r03_parity2.log 2>&1 &&
timeout -k 10 200 tools/gemm_lab > gpurun_out/r03_gemm_lab.txt 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/r03_bench_full.json 2> gpurun_out/r03_bench_full.err &&
FBN_WINDOW_ONEPASS=1 timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_win_one.json 2> gpurun_out/r03_win_one.err &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5.py -x -v --timeout 250 --timeout-method thread > gpurun_out/r03_c5_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --rows-per-gpu 12500000 --no-fp32 --no-cpu-baseline --steps 30 > gpurun_out/r03_c5.json 2> gpurun_out/r03_c5.err &&
timeout -k 10 300 python -u bench.py --rows-per-gpu 12500000 --table-adam sparse --no-fp32 --no-cpu-baseline --steps 30 > gpurun_out/r03_c5_sparse.json 2> gpurun_out/r03_c5_sparse.err
