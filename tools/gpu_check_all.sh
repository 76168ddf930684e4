# Whole-tree check on a fresh box: every GPU test, the default bench line, then a rocprof kernel trace
# of the bench and its step timeline.  Usage (via gpurun): bash tools/gpu_check_all.sh <tag>
set -o pipefail
TAG=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
bash tools/gpu_prof.sh $TAG --no-fp32
