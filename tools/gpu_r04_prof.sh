#!/bin/bash
# Round 4 profiles in one GPU call: the headline bench under rocprofv3 (kernel trace + stats, per-step
# timeline), the one-rank sharded step (kernel trace + host profile), then the PMC passes of the
# headline bench.  Usage (via gpurun): bash tools/gpu_r04_prof.sh <tag>
set -o pipefail
TAG=${1:-r04p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_prof.sh $TAG --no-fp32 --no-inference --no-cpu-plan || exit $?
bash tools/shard_prof.sh ${TAG}_shard || exit $?
cd $R && bash tools/gpu_pmc.sh $TAG || exit $?
