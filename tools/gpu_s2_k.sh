# direct slab sums in the step's deferred-sum launch (FBN_SLAB_DIRECT): trainer / kernel tests, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_kernels.py tests/test_gpu_coverage.py > gpurun_out/s2k_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_step.py base nodirect:env.FBN_SLAB_DIRECT=0 > gpurun_out/s2k_ab.txt 2>&1
