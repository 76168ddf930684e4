# DMA GEMM ring depth: isolated GEMM timings (default plans) and the full bench per setting
R=$GRAFT_REPO_ROOT
for S in 2 3 4; do
  echo "== stages $S"
  FBN_GEMM_STAGES=$S timeout -k 10 200 python $R/tools/gemm_sweep.py F3 dc dWa dW4 F4 > $R/gpurun_out/stage_$S.log 2>&1 || exit 1
  grep dma16 $R/gpurun_out/stage_$S.log | sed 's/best:.*//'
  FBN_GEMM_STAGES=$S timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 40 > $R/gpurun_out/stage_b$S.json 2>/dev/null || exit 1
  grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/stage_b$S.json
done
