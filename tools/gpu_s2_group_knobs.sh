# grouped weight-gradient launch: fewer K-slabs per problem (FBN_GROUP_SPLIT_DIV) and a 3-stage ring
# (FBN_GROUP_STAGES); prefetch entries per wave sized to whole blocks per CU (FBN_PF_EPW 56: 768 blocks
# = 3 per CU; 42: 1024 = 4 per CU; 28: 1536 > the resident slots, dispatched as others finish)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_step.py base div2:env.FBN_GROUP_SPLIT_DIV=2 div4:env.FBN_GROUP_SPLIT_DIV=4 st3:env.FBN_GROUP_STAGES=3 > gpurun_out/s2_gk_ab.txt 2>&1 &&
timeout -k 10 600 python -u tools/ab_step.py base e56:env.FBN_PF_EPW=56 e42:env.FBN_PF_EPW=42 e28:env.FBN_PF_EPW=28 > gpurun_out/s2_epw_ab.txt 2>&1
