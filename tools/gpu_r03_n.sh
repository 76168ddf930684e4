# kernel trace of the default bench (eager, current build) -> verbose step timeline + stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_prof.sh r03n --no-fp32 > gpurun_out/r03n_prof.txt 2>&1 &&
cd $R && python tools/step_timeline.py gpurun_out/prof_r03n/run_kernel_trace.csv --steps 3 --verbose > gpurun_out/timeline_r03n_verbose.txt 2>&1 &&
cp gpurun_out/prof_r03n/run_kernel_stats.csv gpurun_out/r03n_kernel_stats.csv && rm -rf gpurun_out/prof_r03n
