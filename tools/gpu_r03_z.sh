# tiny-output weight-gradient GEMM plan: kernel tests, in-process A/B, C5-shard bench line
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_trainer.py > gpurun_out/r03z_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_step.py base oldtiny:env.FBN_GEMM_TINY=0 > gpurun_out/r03z_ab.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --rows-per-gpu 12500000 --no-cpu-baseline --no-fp32 > gpurun_out/r03z_c5.json 2> gpurun_out/r03z_c5.err
