#!/bin/bash
# Final profiles of the round: rocprofv3 kernel trace + stats of the bench's GPU legs (the driver's
# command minus the CPU / fp32 / inference legs), gzipped trace; then the PMC passes (stdout summary).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04fin; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- \
  python $R/bench.py --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 > $O/c3.log 2>&1 || exit 1
gzip -f $O/c3/run_kernel_trace.csv
cd $R
bash tools/gpu_pmc.sh r04fin > $O/pmc.txt 2>&1 || { tail -20 $O/pmc.txt; exit 1; }
rm -rf $R/gpurun_out/pmc_r04fin/p*
tail -40 $O/pmc.txt
