# Round evidence in one GPU call: tools/gpu_final.sh (every -m gpu test, the default bench line with
# its fp32 / bf16_fwd lines and CPU baseline, the Zipf(1.05) line, a rocprofv3 kernel trace + the
# per-step timeline), then the C2 and C5-shard (lazy, sparse) lines.  Usage: bash tools/gpu_evidence.sh <tag>
set -o pipefail
TAG=${1:-ev}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
bash $R/tools/gpu_final.sh $TAG || exit $?
timeout -k 10 300 python $R/bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 \
  > $OUT/c2_$TAG.json 2> $OUT/c2_$TAG.err || exit 1
echo "c2 $(grep -o '"ms_per_step": [0-9.]*' $OUT/c2_$TAG.json)"
timeout -k 10 400 python $R/bench.py --rows-per-gpu 12500000 --no-cpu-baseline --no-fp32 \
  > $OUT/c5_$TAG.json 2> $OUT/c5_$TAG.err || exit 1
echo "c5 lazy $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5_$TAG.json)"
timeout -k 10 400 python $R/bench.py --rows-per-gpu 12500000 --table-adam sparse --no-cpu-baseline --no-fp32 \
  > $OUT/c5s_$TAG.json 2> $OUT/c5s_$TAG.err || exit 1
echo "c5 sparse $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5s_$TAG.json)"
