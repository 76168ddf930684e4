# full GPU test suite of the current build, kernel trace + step timeline, PMC passes (summaries only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03u_gpu_tests.log 2>&1 &&
bash tools/gpu_prof.sh r03u --no-fp32 > gpurun_out/r03u_prof.txt 2>&1 &&
cd $R && python tools/step_timeline.py gpurun_out/prof_r03u/run_kernel_trace.csv --steps 3 --verbose > gpurun_out/timeline_r03u_verbose.txt 2>&1 &&
cp gpurun_out/prof_r03u/run_kernel_stats.csv gpurun_out/r03u_kernel_stats.csv && rm -rf gpurun_out/prof_r03u &&
PMC_PRIME=64 bash tools/gpu_pmc.sh r03u > gpurun_out/r03u_pmc.txt 2>&1 &&
cd $R && python tools/pmc_traffic.py gpurun_out/pmc_r03u/p3 gpurun_out/pmc_r03u/p4 gpurun_out/r03u_pmc_traffic.json >> gpurun_out/r03u_pmc.txt 2>&1 &&
cp gpurun_out/pmc_r03u/summary.json gpurun_out/r03u_pmc_summary.json && rm -rf gpurun_out/pmc_r03u
