#!/bin/bash
# Round 4 evidence, part 1: the whole -m gpu suite, then the default bench line (driver command), the
# Zipf(1.05) line, the C2 line and the C5-shard lines.  Usage (via gpurun): bash tools/gpu_r04_evidence.sh <tag>
set -o pipefail
TAG=${1:-r04ev}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $R/tests -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench.json | head -1)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python $R/bench.py --no-cpu-baseline --no-fp32 --no-inference --zipf 1.05 > $OUT/bench_zipf.json 2> $OUT/bench_zipf.err
rc=$?; echo "zipf rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_zipf.json | head -1)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python $R/bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 \
  --no-inference > $OUT/c2.json 2> $OUT/c2.err
rc=$?; echo "c2 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/c2.json | head -1)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python $R/bench.py --rows-per-gpu 12500000 --no-cpu-baseline --no-fp32 --no-inference > $OUT/c5.json 2> $OUT/c5.err
rc=$?; echo "c5 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5.json | head -1)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python $R/bench.py --rows-per-gpu 12500000 --table-adam sparse --no-cpu-baseline --no-fp32 --no-inference \
  > $OUT/c5s.json 2> $OUT/c5s.err
rc=$?; echo "c5 sparse rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5s.json | head -1)"; [ $rc -eq 0 ] || exit $rc
FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 timeout -k 10 400 \
  python $R/bench.py --no-cpu-baseline --no-fp32 --no-inference --no-cpu-plan > $OUT/shard.json 2> $OUT/shard.err
rc=$?; echo "shard rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/shard.json | head -1)"; exit $rc
