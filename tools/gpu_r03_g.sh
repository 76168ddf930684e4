# host-side profile of the eager step; rocprofv3 kernel trace + stats of the default bench; PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 200 python -u tools/host_profile.py > gpurun_out/r03_host_profile.txt 2>&1 &&
bash tools/gpu_prof.sh r03 --no-fp32 > gpurun_out/r03_prof.txt 2>&1 &&
PMC_PRIME=64 bash tools/gpu_pmc.sh r03 > gpurun_out/r03_pmc.txt 2>&1 &&
cd $R && python tools/pmc_traffic.py gpurun_out/pmc_r03/p3 gpurun_out/pmc_r03/p4 gpurun_out/r03_pmc_traffic.json >> gpurun_out/r03_pmc.txt 2>&1
