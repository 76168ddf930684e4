# in-process A/B of the stream placement switches (claims / duplicate fold on the side stream)
set -o pipefail
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_trainer.py > gpurun_out/r03p_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_step.py base claim_main:trainer._CLAIM_ON_SIDE=False fixup_main:trainer._FIXUP_ON_SIDE=False both_main:trainer._CLAIM_ON_SIDE=False,trainer._FIXUP_ON_SIDE=False > gpurun_out/r03p_ab.txt 2>&1
