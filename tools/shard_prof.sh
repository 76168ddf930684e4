#!/bin/bash
# The sharded (N > 1) step as a one-rank RCCL job on one GPU: bench line, rocprofv3 kernel trace
# and a host-side cProfile.  Usage (via gpurun): bash tools/shard_prof.sh <tag>
TAG=${1:-sh}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
  python $R/bench.py --gpus 1 --no-fp32 --no-cpu-baseline --steps 20 > $R/gpurun_out/prof_$TAG.log 2>&1 || exit 1
cd $R
timeout -k 10 400 python -m cProfile -o gpurun_out/host_$TAG.prof bench.py --gpus 1 --no-fp32 --no-cpu-baseline \
  > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
python -c "
import pstats; p=pstats.Stats('gpurun_out/host_$TAG.prof'); p.sort_stats('tottime').print_stats(40)" > gpurun_out/host_$TAG.txt
