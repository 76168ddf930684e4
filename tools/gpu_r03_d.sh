# GEMM lab (schedule B) + gather chunk A/B + gather/trainer tests at the new default
set -o pipefail
timeout -k 10 200 tools/gemm_lab > gpurun_out/r03_gemm_lab2.txt 2>&1 &&
for h in 5 10 20 5 10 20; do FBN_FIELDS_HCH=$h timeout -k 10 120 python -u tools/time_fields.py || exit 1; done > gpurun_out/r03_fields_hch.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_fields_tests2.log 2>&1
