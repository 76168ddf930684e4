# the duplicate-gradient fold on the side stream beside the grouped weight-gradient launch
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_step.py base fixside:trainer._FIXUP_ON_SIDE=True > gpurun_out/s2g_ab.txt 2>&1
