#!/bin/bash
# Round evidence in one GPU call: the whole -m gpu suite, the default bench line (with the CPU
# baseline), a rocprofv3 kernel trace + stats of the bench with the per-step timeline, and the
# Zipf(1.05) bench line.  Usage (via gpurun): bash tools/gpu_final.sh <tag>
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $R/tests -q -m gpu -p no:cacheprovider --timeout 180 --timeout-method thread \
  > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python $R/bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python $R/bench.py --no-cpu-baseline --no-fp32 --zipf 1.05 > $OUT/bench_zipf_$TAG.json 2> $OUT/bench_zipf_$TAG.err
rc=$?; echo "bench zipf rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash $R/tools/gpu_prof.sh $TAG --no-fp32 > /dev/null
rc=$?; echo "prof rc=$rc"; exit $rc
