#!/bin/bash
# Round-end evidence in one GPU call: tools/gpu_final.sh (whole -m gpu suite, default bench line,
# Zipf line, rocprofv3 trace + timeline), then the sharded (N > 1) step as a one-rank RCCL job with
# per-GPU and synchronised BatchNorm, then a 4-rank gloo rehearsal of the N > 1 bench path.
# Usage (via gpurun): bash tools/gpu_round_end.sh <tag>
TAG=${1:-end}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
bash $R/tools/gpu_final.sh $TAG || exit $?
for bn in local sync; do
  FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 \
    timeout -k 10 300 python $R/bench.py --gpus 1 --no-fp32 --no-cpu-baseline --bn $bn > $OUT/shard_${bn}_$TAG.json \
    2>/dev/null || exit 1
  echo "shard bn=$bn $(grep -o '"ms_per_step": [0-9.]*' $OUT/shard_${bn}_$TAG.json)"
done
FBN_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29541 $R/bench.py --gpus 4 --no-fp32 --steps 5 --warmup 2 --prime 0 \
  --batches 8 --rows-per-gpu 200000 > $OUT/rehearse4_$TAG.json 2> $OUT/rehearse4_$TAG.err
rc=$?; echo "rehearsal (4 ranks, gloo) rc=$rc"; exit $rc
