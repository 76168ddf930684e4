# row-state record, slab-mode wgrads + one deferred-sum launch, buffer-load gather: tests, bench A/B, PMC
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_trainer.py tests/test_gpu_c5.py tests/test_gpu_multirank.py > gpurun_out/r03h_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err &&
FBN_FIELDS_NOBUF=1 FBN_DEFER_REDUCE=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 > gpurun_out/r03h_bench_old.json 2> gpurun_out/r03h_bench_old.err &&
FBN_FIELDS_NOBUF=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 > gpurun_out/r03h_bench_nobuf.json 2> gpurun_out/r03h_bench_nobuf.err &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 --main-priority > gpurun_out/r03h_bench_prio.json 2> gpurun_out/r03h_bench_prio.err &&
PMC_PRIME=64 bash tools/gpu_pmc.sh r03h > gpurun_out/r03h_pmc.txt 2>&1 &&
python tools/pmc_traffic.py gpurun_out/pmc_r03h/p3 gpurun_out/pmc_r03h/p4 gpurun_out/r03h_pmc_traffic.json >> gpurun_out/r03h_pmc.txt 2>&1 &&
cp gpurun_out/pmc_r03h/summary.json gpurun_out/r03h_pmc_summary.json && rm -rf gpurun_out/pmc_r03h
