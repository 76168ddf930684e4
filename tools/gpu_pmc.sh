#!/bin/bash
# rocprofv3 PMC passes over an eager bench (one pass per counter group; slot limits per pass:
# 8 SQ, 4 TCC, 2 GRBM), then the per-kernel summary.  Usage (via gpurun): bash tools/gpu_pmc.sh <tag>
set -o pipefail
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python $R/bench.py --steps 3 --warmup 1 --prime ${PMC_PRIME:-64} --probe-steps 0 --mode eager --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32"
i=0
PASSES=${PMC_PASSES:-"SQ_WAVES,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,GRBM_GUI_ACTIVE;SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_WAVE_CYCLES,GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE;SQ_WAIT_ANY,SQ_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_LDS"}
IFS=';' read -ra PS <<< "$PASSES"
DIRS=""
for P in "${PS[@]}"; do
  C=${P//,/ }
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/p$i -o run -- $BENCH > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($C) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  DIRS="$DIRS $OUT/p$i"
done
cd $R && python tools/pmc_sq.py $OUT/summary.json $DIRS && \
for d in $DIRS; do gzip -f $d/run_counter_collection.csv; rm -f $d/run_kernel_trace.csv $d/*agent_info.csv; done
