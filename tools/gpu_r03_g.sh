# host-side profile of the eager step; rocprofv3 kernel trace + stats of the default bench; PMC passes
# (large CSVs are summarised on the box and deleted: gpurun_out must stay under 64 MiB)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 200 python -u tools/host_profile.py > gpurun_out/r03_host_profile.txt 2>&1 &&
bash tools/gpu_prof.sh r03 --no-fp32 > gpurun_out/r03_prof.txt 2>&1 &&
cd $R && python tools/step_timeline.py gpurun_out/prof_r03/run_kernel_trace.csv --steps 3 --verbose > gpurun_out/timeline_r03_verbose.txt 2>&1 &&
cp gpurun_out/prof_r03/run_kernel_stats.csv gpurun_out/r03_kernel_stats.csv && rm -rf gpurun_out/prof_r03 &&
PMC_PRIME=64 bash tools/gpu_pmc.sh r03 > gpurun_out/r03_pmc.txt 2>&1 &&
cd $R && python tools/pmc_traffic.py gpurun_out/pmc_r03/p3 gpurun_out/pmc_r03/p4 gpurun_out/r03_pmc_traffic.json >> gpurun_out/r03_pmc.txt 2>&1 &&
cp gpurun_out/pmc_r03/summary.json gpurun_out/r03_pmc_summary.json && rm -rf gpurun_out/pmc_r03
