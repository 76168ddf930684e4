# in-process A/Bs: bf16 image placement, gather chunk, BN apply rows, GEMM tile / ring depth
set -o pipefail
timeout -k 10 500 python -u tools/ab_step.py base w16side:trainer._W16_MODE="'side'" w16late:trainer._W16_MODE="'late'" hch5:env.FBN_FIELDS_HCH=5 hch20:env.FBN_FIELDS_HCH=20 > gpurun_out/r03r_ab1.txt 2>&1 &&
timeout -k 10 500 python -u tools/ab_step.py base rpc8:env.FBN_BN_ACT_RPC=8 big128:env.FBN_DMA_BIG_TILE="'128,128'" stages3:env.FBN_GEMM_STAGES=3 > gpurun_out/r03r_ab2.txt 2>&1
