# grouped weight-gradient GEMMs (FBN_WGRAD_GROUP) and the step head (claims + bf16 images in one launch,
# FBN_HEAD_CONV): bit-identity + the trainer / kernel tests, then the in-process A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_kernels.py > gpurun_out/s2_wg_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_step.py base nogroup:ops._WGRAD_GROUP=False nohead:trainer._HEAD_CONV=False neither:ops._WGRAD_GROUP=False\;trainer._HEAD_CONV=False > gpurun_out/s2_wg_ab.txt 2>&1
