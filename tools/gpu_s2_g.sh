# replay group size (FBN_PF_G / FBN_WIN_G = 2: half the side-stream register footprint): bit-identity, then A/B
set -o pipefail
mkdir -p gpurun_out
FBN_PF_G=2 FBN_WIN_G=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trainer.py -k "prefetch or lazy or window" > gpurun_out/s2_g_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_step.py base pg2:env.FBN_PF_G=2 wg2:env.FBN_WIN_G=2 both:env.FBN_PF_G=2\;env.FBN_WIN_G=2 both_e32:env.FBN_PF_G=2\;env.FBN_WIN_G=2\;env.FBN_PF_EPW=32 > gpurun_out/s2_g_ab.txt 2>&1
