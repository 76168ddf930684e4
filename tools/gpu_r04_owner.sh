#!/bin/bash
# Two-pass owner-side prefetch (N > 1 row-sharded steps): bit-identity + multirank/RCCL tests, then the
# one-rank sharded bench with FBN_OWNER_PF2=1 (two-pass, default) and =0 (one-pass), and a kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04own; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_multirank.py tests/test_gpu_rccl.py "tests/test_gpu_trainer.py::test_next_batch_prefetch_bit_identical" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
export FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
for pf in 1 0; do
  FBN_OWNER_PF2=$pf timeout -k 10 300 python bench.py --gpus 1 --no-fp32 --no-cpu-baseline --no-cpu-plan --no-inference \
    > $O/bench_pf2_$pf.json 2> $O/bench_pf2_$pf.err || exit 1
  tail -1 $O/bench_pf2_$pf.json | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python $R/bench.py --gpus 1 --no-fp32 --no-cpu-baseline --no-cpu-plan --no-inference --steps 20 > $O/prof.log 2>&1 || exit 1
cd $R && python tools/step_timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt 2>&1; head -40 $O/timeline.txt
