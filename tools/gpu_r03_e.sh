# BN1 backward partials in the dgrad GEMM epilogue: tests + bench A/B; F3 GEMM forms vs lab on one box
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_trainer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_bn1_tests.log 2>&1 &&
FBN_PARITY_OUT=gpurun_out/parity timeout -k 10 500 python -u -m pytest tests/test_gpu_coverage.py -x -q -s --timeout 400 --timeout-method thread -k "precision_modes and small" > gpurun_out/r03_bn1_parity.log 2>&1 &&
timeout -k 10 120 python -u tools/gemm_f3.py > gpurun_out/r03_gemm_f3.txt 2>&1 &&
timeout -k 10 200 tools/gemm_lab > gpurun_out/r03_gemm_lab3.txt 2>&1 &&
FBN_BN1_BWD_IN_GEMM=0 timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_bn1_off.json 2> gpurun_out/r03_bn1_off.err &&
timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_bn1_on.json 2> gpurun_out/r03_bn1_on.err &&
FBN_BN1_BWD_IN_GEMM=0 timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_bn1_off2.json 2> gpurun_out/r03_bn1_off2.err &&
timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_bn1_on2.json 2> gpurun_out/r03_bn1_on2.err
