# PMC passes of the default bench (tools/gpu_pmc.sh), then the per-launch HBM bytes of the roofline
# kernels; the raw pass directories are removed afterwards (gpurun copies back at most 64 MiB)
set -o pipefail
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_pmc.sh $TAG || exit $?
cd $R && python tools/pmc_traffic.py gpurun_out/pmc_$TAG/p3 gpurun_out/pmc_$TAG/p4 gpurun_out/pmc_$TAG/traffic.json || exit 1
rm -rf gpurun_out/pmc_$TAG/p[0-9]*
