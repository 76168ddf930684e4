# this session's step changes: grouped weight gradients (FBN_WGRAD_GROUP, FBN_GROUP_SPLIT_DIV), the step
# head (FBN_HEAD_CONV), the window in the prefetch's launch (FBN_PF_WINDOW): trainer / kernel tests, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_kernels.py > gpurun_out/s2_wg_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_step.py base nomerge:trainer._PF_WINDOW=False div1:env.FBN_GROUP_SPLIT_DIV=1 div3:env.FBN_GROUP_SPLIT_DIV=3 > gpurun_out/s2_wg_ab2.txt 2>&1
