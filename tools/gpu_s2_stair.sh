# replay engine staircase: all GPU tests, the prefetch ablation, the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2c_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/pf_ablation.py > gpurun_out/s2c_pfabl.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-fp32 > gpurun_out/s2c_bench.json 2> gpurun_out/s2c_bench.err
