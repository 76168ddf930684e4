# GEMM ring depth x tile plans on the large C3 shapes, with hipBLASLt (torch.mm) as a reference point
R=$GRAFT_REPO_ROOT
for S in ${STAGES:-2 3 4}; do
  echo "== stages $S"
  FBN_SWEEP_DMA_ONLY=1 FBN_GEMM_STAGES=$S timeout -k 10 300 python $R/tools/gemm_sweep.py ${SHAPES:-F3 dc dWa U F4 dh1 dW4} > $R/gpurun_out/gprobe_$S.log 2>&1 || exit 1
  grep dma16 $R/gpurun_out/gprobe_$S.log
done
