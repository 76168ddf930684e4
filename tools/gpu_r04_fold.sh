#!/bin/bash
# Owner gradient fold (fbn_owner_claim lists + fbn_owner_grad): unit test, sharded parity tests, then the
# one-rank sharded bench and its kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04fold; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_exchange.py \
  tests/test_gpu_rccl.py tests/test_gpu_multirank.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
export FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 300 python bench.py --gpus 1 --no-fp32 --no-cpu-baseline --no-cpu-plan --no-inference \
  > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python $R/bench.py --gpus 1 --no-fp32 --no-cpu-baseline --no-cpu-plan --no-inference --steps 20 > $O/prof.log 2>&1 || exit 1
