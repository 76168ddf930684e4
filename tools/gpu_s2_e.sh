# prefetch ablation with 8-row groups; the 256 x 256 bf16-output dgrad tile (FBN_BF16OUT_TILE): its test, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pf_ablation.py > gpurun_out/s2d_pfabl.txt 2>&1 &&
FBN_BF16OUT_TILE=256 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "bf16out" > gpurun_out/s2e_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_step.py base t256:env.FBN_BF16OUT_TILE=256 > gpurun_out/s2e_ab.txt 2>&1
