# tests -> A/B bench vs tools/variants/prev -> rocprof kernel trace of this tree's bench
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
ROUNDS=${2:-2}
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest $R/tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $R/gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -15 $R/gpurun_out/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash $R/tools/ab.sh $ROUNDS || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
  python $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
