#!/bin/bash
# Round 4 evidence, part 2: rocprofv3 kernel trace + stats of the bench (the driver's command minus
# the CPU legs) with the per-step timeline, the PMC passes of the headline step, the C2 trace.
set -o pipefail
TAG=${1:-r04prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_prof.sh $TAG --no-inference --no-cpu-plan > /dev/null || exit $?
bash tools/gpu_pmc.sh $TAG || exit $?
bash tools/gpu_prof.sh ${TAG}_c2 --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-fp32 --no-inference --no-cpu-plan > /dev/null || exit $?
