# GEMM lab (schedule B) + gather chunk A/B + engine tests (d = 16 / 64 / 128 / 256) + C2 bench and trace
set -o pipefail
timeout -k 10 200 tools/gemm_lab > gpurun_out/r03_gemm_lab2.txt 2>&1 &&
for h in 5 10 20 5 10 20; do FBN_FIELDS_HCH=$h timeout -k 10 120 python -u tools/time_fields.py || exit 1; done > gpurun_out/r03_fields_hch.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_trainer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_engine_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-fp32 --no-cpu-baseline --steps 30 > gpurun_out/r03_c2b.json 2> gpurun_out/r03_c2b.err &&
bash tools/gpu_prof.sh c2 --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-fp32
