#!/bin/bash
# One GPU-box session: gpu tests -> bench -> rocprofv3 kernel trace of a short bench.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh <tag> [tests|bench|prof]...
set -o pipefail
TAG=${1:-r1}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 1000 python -u -m pytest $R/tests -v -m gpu -p no:cacheprovider --timeout 180 --timeout-method thread \
        > $OUT/tests_$TAG.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -5 $OUT/tests_$TAG.log
      # rc 1 = test failures (keep going); anything else (timeout, crash, fault) ends the session
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    bench)
      timeout -k 10 900 python $R/bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
      rc=$?; echo "bench rc=$rc"; cat $OUT/bench_$TAG.json; tail -5 $OUT/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc ;;
    benchfast)
      timeout -k 10 600 python $R/bench.py --no-cpu-baseline > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
      rc=$?; echo "bench rc=$rc"; cat $OUT/bench_$TAG.json; tail -5 $OUT/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
        python $R/bench.py --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -3 $OUT/prof_$TAG.log; cd $R; [ $rc -eq 0 ] || exit $rc ;;
    pmc)
      cd /tmp && export TMPDIR=/tmp
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_${TAG}_$C -o run -- \
          python $R/bench.py --steps 4 --warmup 2 --probe-steps 1 --no-graph --no-cpu-baseline > $OUT/pmc_${TAG}_$C.log 2>&1
        rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done
      cd $R ;;
  esac
done
# (appended) PMC traffic passes: FETCH_SIZE and WRITE_SIZE in separate runs (slot limits)
