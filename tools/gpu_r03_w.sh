# host-side trims (cached scratch, bound ctypes functions): GPU tests, host profile, C2 / C3 GPU-bound vs live
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03w_gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/host_profile.py > gpurun_out/r03w_host_profile.txt 2>&1 &&
EG_D=16 EG_V=1000000 EG_B=4096 timeout -k 10 200 python -u tools/eager_gpu_time.py > gpurun_out/r03w_c2_gpu.txt 2>&1 &&
timeout -k 10 200 python -u tools/eager_gpu_time.py > gpurun_out/r03w_c3_gpu.txt 2>&1 &&
timeout -k 10 200 python -u bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 > gpurun_out/r03w_c2.json 2> gpurun_out/r03w_c2.err
