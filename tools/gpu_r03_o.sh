# end-aligned replay engine with scalar constants, unrolled step tail + two-level ticket, claims on
# the side stream: lazy-Adam bit-identity tests, bench A/Bs, PMC of the replay kernels
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_c5.py tests/test_gpu_multirank.py tests/test_gpu_kernels.py > gpurun_out/r03o_tests.log 2>&1 &&
for rnd in 1 2; do
  for cfg in "X=0" "FBN_CLAIM_ON_SIDE=0" "FBN_PF_EPW=16"; do
    tag=$(echo $cfg | tr -d ' =_' | tr 'A-Z' 'a-z')
    env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 > gpurun_out/r03o_bench_${tag}_$rnd.json 2> gpurun_out/r03o_bench_${tag}_$rnd.err || exit 1
  done
done &&
PMC_PRIME=64 PMC_PASSES="SQ_WAVES,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE" bash tools/gpu_pmc.sh r03o > gpurun_out/r03o_pmc.txt 2>&1 &&
python tools/pmc_traffic.py gpurun_out/pmc_r03o/p2 gpurun_out/pmc_r03o/p3 gpurun_out/r03o_pmc_traffic.json >> gpurun_out/r03o_pmc.txt 2>&1 &&
cp gpurun_out/pmc_r03o/summary.json gpurun_out/r03o_pmc_summary.json && rm -rf gpurun_out/pmc_r03o
