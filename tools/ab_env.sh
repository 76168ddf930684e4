# A/B bench within one tree: env setting A vs B, alternating.  bash tools/ab_env.sh rounds "VAR=a" "VAR=b"
R=$GRAFT_REPO_ROOT
N=${1:-3}; A=$2; B=$3
for i in $(seq 1 $N); do
  for e in "$A" "$B"; do
    env $e timeout -k 10 200 python $R/bench.py --no-cpu-baseline > $R/gpurun_out/abe_$i.json 2>/dev/null || exit 1
    echo "[$e] $i $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/abe_$i.json)"
  done
done
