# hot-row staging A/B (N1) + buffer-load gather A/B, uniform and Zipf(1.05); hot-staging tests
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r03i_tests.log 2>&1 &&
for z in 0 1.05; do
  for cfg in "" "FBN_FIELDS_NOBUF=1" "FBN_GATHER_HOT=2" "FBN_GATHER_HOT=4" "FBN_GATHER_HOT=8"; do
    env ZIPF=$z $cfg timeout -k 10 120 python -u tools/time_fields.py >> gpurun_out/r03i_fields.txt 2>&1 || exit 1
  done
done &&
timeout -k 10 200 python -u bench.py --zipf 1.05 --no-cpu-baseline --no-fp32 > gpurun_out/r03i_bench_zipf.json 2> gpurun_out/r03i_bench_zipf.err &&
FBN_GATHER_HOT=4 timeout -k 10 200 python -u bench.py --zipf 1.05 --no-cpu-baseline --no-fp32 > gpurun_out/r03i_bench_zipf_hot4.json 2> gpurun_out/r03i_bench_zipf_hot4.err
