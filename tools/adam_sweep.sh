# untouched-Adam workgroup throttle sweep (bench ms/step per setting)
R=$GRAFT_REPO_ROOT
for nb in 128 256 384 512 1024; do
  FBN_ADAM_BLOCKS=$nb timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 40 > $R/gpurun_out/adam_$nb.json 2>/dev/null || exit 1
  echo "$nb $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/adam_$nb.json) $(grep -o '"avg_launch_ms": [0-9.]*' $R/gpurun_out/adam_$nb.json | head -1)"
done
