#!/bin/bash
# Early gradient exchange with native RCCL (the gradient-row all-to-all on the exchange's own stream,
# beside the grouped weight gradients): the RCCL test, then the one-rank sharded line with and without.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04early; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rccl.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 FBN_BENCH_SHARD=1
for rnd in 1 2; do
  for e in 1 0; do
    FBN_EARLY_GRAD_XCHG=$e MASTER_PORT=2957$rnd timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32 --no-inference \
      --no-cpu-plan > $O/early${e}_$rnd.json 2> $O/early${e}_$rnd.err || { tail -20 $O/early${e}_$rnd.err; exit 1; }
    echo "early=$e $rnd $(grep -o '"ms_per_step": [0-9.]*' $O/early${e}_$rnd.json | head -1)"
  done
done
