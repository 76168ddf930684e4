# tests of the reworked deferred-sum / commit kernels, a step timeline, the bench line, C2 GPU-bound time
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_kernels.py tests/test_gpu_multirank.py > gpurun_out/r03v_tests.log 2>&1 &&
bash tools/gpu_prof.sh r03v --no-fp32 > gpurun_out/r03v_prof.txt 2>&1 &&
cd $R && python tools/step_timeline.py gpurun_out/prof_r03v/run_kernel_trace.csv --steps 3 --verbose > gpurun_out/timeline_r03v_verbose.txt 2>&1 &&
rm -rf gpurun_out/prof_r03v &&
timeout -k 10 300 python -u bench.py > gpurun_out/r03v_bench.json 2> gpurun_out/r03v_bench.err &&
EG_D=16 EG_V=1000000 EG_B=4096 timeout -k 10 200 python -u tools/eager_gpu_time.py > gpurun_out/r03v_c2_gpu.txt 2>&1
