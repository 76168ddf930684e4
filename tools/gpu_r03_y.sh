# side-stream footprint caps (grid-strided prefetch / window with few waves): tests with caps on, A/B
set -o pipefail
FBN_PF_WAVES=1024 FBN_WIN_WAVES=512 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trainer.py -k "prefetch or lazy or interleave" > gpurun_out/r03y_tests_caps.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_c5.py > gpurun_out/r03y_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_step.py base pf1024:env.FBN_PF_WAVES=1024 pf2048:env.FBN_PF_WAVES=2048 pf512:env.FBN_PF_WAVES=512 win512:env.FBN_WIN_WAVES=512 both:env.FBN_PF_WAVES=1024\;env.FBN_WIN_WAVES=512 > gpurun_out/r03y_ab.txt 2>&1
