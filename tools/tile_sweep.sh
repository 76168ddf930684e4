# large-output GEMM tile under the overlapped Adam: bench ms/step per tile
R=$GRAFT_REPO_ROOT
for t in 64,64 128,64 64,128 128,128; do
  FBN_DMA_BIG_TILE=$t timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 40 > $R/gpurun_out/tile_$t.json 2>/dev/null || exit 1
  echo "$t $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/tile_$t.json)"
done
