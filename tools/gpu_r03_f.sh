# fast GEMM epilogue + graph/eager interleave test + launch-mode trial bench
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_trainer.py tests/test_gpu_coverage.py -x -q --timeout 250 --timeout-method thread -k "not precision_modes" > gpurun_out/r03_f_tests.log 2>&1 &&
timeout -k 10 120 python -u tools/gemm_f3.py > gpurun_out/r03_gemm_f3b.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_auto1.json 2> gpurun_out/r03_auto1.err &&
timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 --mode graph > gpurun_out/r03_graph1.json 2> gpurun_out/r03_graph1.err &&
timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_auto2.json 2> gpurun_out/r03_auto2.err
