#!/bin/bash
# The N > 1 code paths on a one-GPU box: the multi-rank and RCCL GPU tests, then the sharded step
# as a one-rank RCCL job with per-GPU and synchronised BatchNorm, then a 2-rank gloo rehearsal of
# the bench (correctness of the N > 1 bench path; its timing means nothing).
# Usage (via gpurun): bash tools/gpu_shard_ab.sh <tag>
TAG=${1:-sh}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $R/tests/test_gpu_multirank.py $R/tests/test_gpu_rccl.py -q -x -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for bn in local sync local sync; do
  FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 \
    timeout -k 10 300 python $R/bench.py --gpus 1 --no-fp32 --no-cpu-baseline --bn $bn > $OUT/shard_$bn.json 2>/dev/null \
    || exit 1
  echo "shard bn=$bn $(grep -o '"ms_per_step": [0-9.]*' $OUT/shard_$bn.json)"
done
FBN_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 $R/bench.py --gpus 2 --no-fp32 --steps 5 --warmup 2 --prime 0 \
  --batches 8 --rows-per-gpu 200000 > $OUT/rehearse_$TAG.json 2> $OUT/rehearse_$TAG.err
rc=$?; echo "rehearsal rc=$rc"; grep -o '"ms_per_step": [0-9.]*\|"batchnorm": "[^"]*"' $OUT/rehearse_$TAG.json; exit $rc
