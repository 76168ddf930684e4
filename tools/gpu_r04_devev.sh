#!/bin/bash
# Device-scope events for the eager steps' stream edges (FBN_DEV_EVENTS): the whole -m gpu suite, then
# the one-rank sharded line and the eager C3 line with and without them, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04devev; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -q -m gpu tests -p no:cacheprovider --timeout 600 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -le 1 ] || exit $rc
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
for rnd in 1 2; do
  for de in 1 0; do
    FBN_DEV_EVENTS=$de FBN_BENCH_SHARD=1 MASTER_PORT=2955$rnd timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32 \
      --no-inference --no-cpu-plan > $O/shard_${de}_$rnd.json 2> $O/shard_${de}_$rnd.err || { tail -20 $O/shard_${de}_$rnd.err; exit 1; }
    echo "shard dev_events=$de $rnd $(grep -o '"ms_per_step": [0-9.]*' $O/shard_${de}_$rnd.json | head -1)"
  done
done
unset RANK WORLD_SIZE LOCAL_RANK
for de in 1 0; do
  FBN_DEV_EVENTS=$de timeout -k 10 300 python bench.py --mode eager --no-cpu-baseline --no-fp32 --no-inference --no-cpu-plan \
    > $O/eager_$de.json 2> $O/eager_$de.err || { tail -20 $O/eager_$de.err; exit 1; }
  echo "c3 eager dev_events=$de $(grep -o '"ms_per_step": [0-9.]*' $O/eager_$de.json | head -1)"
done
