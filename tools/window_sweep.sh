# lazy-Adam rolling-window pass on the side stream: workgroup cap -> bench ms/step
R=$GRAFT_REPO_ROOT
for nb in ${NBS:-64 128 256 512}; do
  FBN_WINDOW_BLOCKS=$nb timeout -k 10 200 python $R/bench.py --no-cpu-baseline > $R/gpurun_out/win_$nb.json 2>/dev/null || exit 1
  echo "$nb $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/win_$nb.json)"
done
