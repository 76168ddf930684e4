#!/bin/bash
# The sharded step as a one-rank RCCL job, interleaved env arms.  Usage (via gpurun):
# bash tools/gpu_shard_arms.sh <tag> <rounds> "" "VAR=a" ...   (runs the N > 1 GPU tests first)
TAG=$1; N=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $R/tests/test_gpu_multirank.py $R/tests/test_gpu_rccl.py -q -x -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq 1 $N); do
  for e in "$@"; do
    (export FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 $e;
     timeout -k 10 300 python $R/bench.py --gpus 1 --no-fp32 --no-cpu-baseline > $OUT/sharm.json 2>/dev/null) || exit 1
    echo "arm [$e] round $i $(grep -o '"ms_per_step": [0-9.]*\|"host_[a-z_]*": [0-9.]*' $OUT/sharm.json | tr '\n' ' ')"
  done
done
