#!/bin/bash
# RCCL on the step's stream (csrc/comm.cpp): the one-rank RCCL parity test, then the one-rank sharded
# bench with FBN_NATIVE_COMM=1 (default) and =0 (torch.distributed), and a kernel trace of the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04nat; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rccl.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
export FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
for nc in 1 0; do
  FBN_NATIVE_COMM=$nc timeout -k 10 300 python bench.py --gpus 1 --no-fp32 --no-cpu-baseline --no-cpu-plan --no-inference \
    > $O/bench_nc$nc.json 2> $O/bench_nc$nc.err || { tail -20 $O/bench_nc$nc.err; exit 1; }
  tail -1 $O/bench_nc$nc.json | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python $R/bench.py --gpus 1 --no-fp32 --no-cpu-baseline --no-cpu-plan --no-inference --steps 20 > $O/prof.log 2>&1 || exit 1
