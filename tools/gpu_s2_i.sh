# grouped weight gradients on 256 x 128 tiles (FBN_GROUP_TILE=256): slab bit-identity, then A/B with half / all slabs
set -o pipefail
mkdir -p gpurun_out
FBN_GROUP_TILE=256 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "slabs_group" tests/test_gpu_trainer.py -k "wgrad_group or slabs_group" > gpurun_out/s2i_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_step.py base t256d1:env.FBN_GROUP_TILE=256\;env.FBN_GROUP_SPLIT_DIV=1 t256d2:env.FBN_GROUP_TILE=256 > gpurun_out/s2i_ab.txt 2>&1
