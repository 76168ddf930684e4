# the N > 1 path on this tree: the sharded step as a one-rank RCCL job (both BatchNorm modes) and a 4-rank
# gloo rehearsal of the N > 1 bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
for bn in local sync; do
  FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 \
    timeout -k 10 300 python $R/bench.py --gpus 1 --no-fp32 --no-cpu-baseline --bn $bn > $OUT/shard_${bn}_s2p.json \
    2> $OUT/shard_${bn}_s2p.err || exit 1
  echo "shard bn=$bn $(grep -o '"ms_per_step": [0-9.]*' $OUT/shard_${bn}_s2p.json)"
done
FBN_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29541 $R/bench.py --gpus 4 --no-fp32 --steps 5 --warmup 2 --prime 0 \
  --batches 8 --rows-per-gpu 200000 > $OUT/rehearse4_s2p.json 2> $OUT/rehearse4_s2p.err
rc=$?; echo "rehearsal (4 ranks, gloo) rc=$rc"; exit $rc
