#!/bin/bash
# rocprofv3 PMC passes over one GEMM shape (tools/gemm_one.py), one pass per counter group, then
# the per-kernel summary (tools/pmc_sq.py).  Usage (via gpurun): bash tools/gemm_pmc.sh <tag> <shape> [iters]
set -o pipefail
TAG=$1; SHAPE=$2; IT=${3:-30}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gpmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PASSES=${PMC_PASSES:-"SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE;SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS;SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_LDS,SQ_LDS_IDX_ACTIVE;TCC_HIT_sum,TCC_MISS_sum;FETCH_SIZE"}
IFS=';' read -ra PS <<< "$PASSES"
DIRS=""
i=0
for P in "${PS[@]}"; do
  C=${P//,/ }
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/p$i -o run -- python $R/tools/gemm_one.py $SHAPE $IT > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($C) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  DIRS="$DIRS $OUT/p$i"
done
cd $R && python tools/pmc_sq.py $OUT/summary.json $DIRS
