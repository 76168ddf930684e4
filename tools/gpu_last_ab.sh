# gather history rows in flight per chunk (FBN_FIELDS_HCH, default 10): a longer in-process A/B
set -o pipefail
mkdir -p gpurun_out
AB_R=10 timeout -k 10 800 python -u tools/ab_step.py base hch5:env.FBN_FIELDS_HCH=5 hch20:env.FBN_FIELDS_HCH=20 > gpurun_out/s2s_ab.txt 2>&1
