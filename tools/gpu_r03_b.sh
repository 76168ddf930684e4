# precision-mode parity (recorded), the full bench line (bf16 + fp32 + bf16_fwd + CPU baseline), window A/B
set -o pipefail
mkdir -p gpurun_out/parity
FBN_PARITY_OUT=gpurun_out/parity timeout -k 10 500 python -u -m pytest tests/test_gpu_coverage.py -x -v -s --timeout 400 --timeout-method thread -k "precision_modes or trainer_step" > gpurun_out/r03_parity.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/r03_bench_full.json 2> gpurun_out/r03_bench_full.err &&
FBN_WINDOW_ONEPASS=1 timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_win_one.json 2> gpurun_out/r03_win_one.err
