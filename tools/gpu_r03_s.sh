# in-process A/B: step-tail block caps; bench line of the current build
set -o pipefail
timeout -k 10 500 python -u tools/ab_step.py base nd512:env.FBN_TAIL_ND=512 nd1024:env.FBN_TAIL_ND=1024 nc1024:env.FBN_TAIL_NC=1024 both1024:env.FBN_TAIL_ND=1024\;env.FBN_TAIL_NC=1024 > gpurun_out/r03s_ab.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r03s_bench.json 2> gpurun_out/r03s_bench.err &&
AB_ZIPF=1.05 timeout -k 10 500 python -u tools/ab_step.py base rpw4:env.FBN_WIN_RPW=4 rpw2:env.FBN_WIN_RPW=2 epw32:env.FBN_PF_EPW=32 > gpurun_out/r03s_ab_zipf.txt 2>&1
