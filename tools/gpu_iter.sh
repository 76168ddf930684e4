#!/bin/bash
# One iteration on the GPU box: the whole -m gpu suite, an interleaved env A/B of the bench
# (arms as in ab_arms.sh), then a rocprofv3 kernel trace + per-step timeline of the default arm.
# Usage (via gpurun): bash tools/gpu_iter.sh <tag> <rounds> "" "VAR=a" ...
TAG=$1; N=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $R/tests -q -m gpu -x -p no:cacheprovider --timeout 180 --timeout-method thread \
  > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash $R/tools/ab_arms.sh $N "$@" || exit 1
bash $R/tools/gpu_prof.sh $TAG --no-fp32 > /dev/null
rc=$?; echo "prof rc=$rc"; head -4 $OUT/timeline_$TAG.txt; exit $rc
