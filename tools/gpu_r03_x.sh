# side-stream pass order A/B (window then prefetch / prefetch then window / window beside the backward)
set -o pipefail
FBN_SIDE_ORDER=p_w timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trainer.py -k "prefetch or lazy or interleave" > gpurun_out/r03x_tests_pw.log 2>&1 &&
timeout -k 10 500 python -u tools/ab_step.py base pw:trainer._SIDE_ORDER="'pw'" p_w:trainer._SIDE_ORDER="'p_w'" > gpurun_out/r03x_ab.txt 2>&1 &&
AB_ZIPF=1.05 timeout -k 10 500 python -u tools/ab_step.py base pw:trainer._SIDE_ORDER="'pw'" p_w:trainer._SIDE_ORDER="'p_w'" > gpurun_out/r03x_ab_zipf.txt 2>&1
