# the d-dependent default lazy window: every GPU test, then the C2 and C3 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2n_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 > gpurun_out/s2n_c2.json 2> gpurun_out/s2n_c2.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32 > gpurun_out/s2n_c3.json 2> gpurun_out/s2n_c3.err
