# trainer / kernel tests of the current build, then the in-process A/Bs and a bench line
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_kernels.py tests/test_gpu_c5.py > gpurun_out/r03t_tests.log 2>&1 &&
timeout -k 10 500 python -u tools/ab_step.py base w16side:trainer._W16_MODE="'side'" w16late:trainer._W16_MODE="'late'" hch5:env.FBN_FIELDS_HCH=5 hch20:env.FBN_FIELDS_HCH=20 > gpurun_out/r03r_ab1.txt 2>&1 &&
timeout -k 10 500 python -u tools/ab_step.py base rpc8:env.FBN_BN_ACT_RPC=8 big128:env.FBN_DMA_BIG_TILE="'128,128'" stages3:env.FBN_GEMM_STAGES=3 > gpurun_out/r03r_ab2.txt 2>&1 &&
timeout -k 10 500 python -u tools/ab_step.py base nd512:env.FBN_TAIL_ND=512 nd1024:env.FBN_TAIL_ND=1024 nc1024:env.FBN_TAIL_NC=1024 both1024:env.FBN_TAIL_ND=1024\;env.FBN_TAIL_NC=1024 > gpurun_out/r03s_ab.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r03s_bench.json 2> gpurun_out/r03s_bench.err &&
AB_ZIPF=1.05 timeout -k 10 500 python -u tools/ab_step.py base rpw4:env.FBN_WIN_RPW=4 rpw2:env.FBN_WIN_RPW=2 epw32:env.FBN_PF_EPW=32 > gpurun_out/r03s_ab_zipf.txt 2>&1
