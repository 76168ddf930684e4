# the merged step head below d = 128: trainer / kernel / coverage tests, then two C2 lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_kernels.py tests/test_gpu_coverage.py tests/test_gpu_parity.py > gpurun_out/s2o_tests.log 2>&1 &&
for r in 1 2; do timeout -k 10 300 python -u bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32 > gpurun_out/s2o_c2_$r.json 2> gpurun_out/s2o_c2_$r.err || exit 1; python -c "import json;d=json.load(open('gpurun_out/s2o_c2_$r.json'));print('C2', d['ms_per_step'], d['config']['hipgraph'])"; done
