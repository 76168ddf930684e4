#!/bin/bash
# One-rank sharded step: kernel + HIP runtime trace (host enqueue times vs kernel starts).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04sht; mkdir -p $O
export FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/prof -o run -- \
  python $R/bench.py --gpus 1 --no-fp32 --no-cpu-baseline --no-cpu-plan --no-inference --steps 10 --warmup 5 \
  > $O/prof.log 2>&1 || exit 1
ls -la $O/prof
