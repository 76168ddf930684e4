#!/bin/bash
# Kernel-span probes (every launch through hipExtLaunchKernelGGL): kernel / program / trainer tests, the
# default bench line, and a kernel trace of the same bench for the roofline-vs-rocprof comparison.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04probe; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_program.py tests/test_gpu_trainer.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench $(grep -o '"ms_per_step": [0-9.]*' $O/bench.json | head -1)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- \
  python $R/bench.py --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 > $O/c3.log 2>&1 || exit 1
gzip -f $O/c3/run_kernel_trace.csv
