#!/bin/bash
# Kernel-span probes recorded into one step program in eight (in-step rooflines from the timed
# replays): the bench with and without them, interleaved, and a rocprof stats run of the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04live2}; mkdir -p $O
cd $R
for rnd in 1 2; do
  for lp in live nolive; do
    F=""; [ $lp = nolive ] && F="--no-live-probes"
    timeout -k 10 400 python bench.py --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 $F > $O/${lp}_$rnd.json \
      2> $O/${lp}_$rnd.err || { tail -20 $O/${lp}_$rnd.err; exit 1; }
    echo "$lp $rnd $(grep -o '"ms_per_step": [0-9.]*' $O/${lp}_$rnd.json | head -1)"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- \
  python $R/bench.py --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 > $O/c3.log 2>&1 || exit 1
rm -f $O/c3/run_kernel_trace.csv
