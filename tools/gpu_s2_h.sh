# side-stream order re-measured on this tree: window then prefetch (default), prefetch then window,
# the window held back until the backward starts
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_step.py base pw:trainer._SIDE_ORDER=\"pw\" p_w:trainer._SIDE_ORDER=\"p_w\" > gpurun_out/s2h_ab.txt 2>&1
