# in-process A/Bs: deferred reduces, side-stream placement / serial, prefetch entries per wave, window rows per wave
set -o pipefail
timeout -k 10 500 python -u tools/ab_step.py base serial:trainer._SIDE_SERIAL=True noslab:ops._DEFER_REDUCE=False mmproj:trainer._SIDE_AFTER_MMPROJ=True mlp0:trainer._SIDE_AFTER_MLP0=True > gpurun_out/r03q_ab1.txt 2>&1 &&
timeout -k 10 500 python -u tools/ab_step.py base epw16:env.FBN_PF_EPW=16 epw64:env.FBN_PF_EPW=64 rpw4:env.FBN_WIN_RPW=4 rpw16:env.FBN_WIN_RPW=16 > gpurun_out/r03q_ab2.txt 2>&1
