#!/bin/bash
# rocprofv3 kernel trace + stats of the default bench command, then the per-step timeline.
# Usage (via gpurun): bash tools/gpu_prof.sh <tag> [bench args...]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
  python $R/bench.py --no-cpu-baseline --steps 20 "$@" > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python tools/step_timeline.py $(ls gpurun_out/prof_$TAG/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof_$TAG/run_kernel_trace.csv) --steps 3 > gpurun_out/timeline_$TAG.txt
echo "timeline rc=$?"; head -40 gpurun_out/timeline_$TAG.txt
