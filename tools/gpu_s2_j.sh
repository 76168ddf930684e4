# XCD-aware block order in the grouped weight-gradient launch (FBN_GROUP_XCD): slab tests, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "slabs_group" tests/test_gpu_trainer.py -k "wgrad_group or slabs_group" > gpurun_out/s2j_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_step.py base noxcd:env.FBN_GROUP_XCD=0 > gpurun_out/s2j_ab.txt 2>&1
