# A/B bench: tools/variants/prev (an older tree with its own built .so) vs this tree, alternating.
#   bash tools/ab.sh [rounds] [extra bench args]
R=$GRAFT_REPO_ROOT
N=${1:-3}; shift
for i in $(seq 1 $N); do
  for t in prev cur; do
    if [ $t = prev ]; then D=$R/tools/variants/prev; else D=$R; fi
    timeout -k 10 200 python $D/bench.py --no-cpu-baseline "$@" > $R/gpurun_out/ab_${t}_$i.json 2>/dev/null || exit 1
    echo "$t $i $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/ab_${t}_$i.json)"
  done
done
