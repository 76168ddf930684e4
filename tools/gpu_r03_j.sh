# replay-engine occupancy A/B (prefetch entries per wave, window rows per wave) + hot-gather kernel A/B
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trainer.py -k "prefetch or lazy or deferred or interleave" > gpurun_out/r03j_tests.log 2>&1 &&
timeout -k 10 120 python -u tools/ab_hot_gather.py 1.05 2 4 8 16 > gpurun_out/r03j_hot_ab.txt 2>&1 &&
timeout -k 10 120 python -u tools/ab_hot_gather.py 0 2 > gpurun_out/r03j_hot_ab_uniform.txt 2>&1 &&
for cfg in "FBN_PF_EPW=64 FBN_WIN_RPW=16" "FBN_PF_EPW=32 FBN_WIN_RPW=8" "FBN_PF_EPW=16 FBN_WIN_RPW=4"; do
  tag=$(echo $cfg | tr -d ' =_A-Z')
  env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 > gpurun_out/r03j_bench_$tag.json 2> gpurun_out/r03j_bench_$tag.err || exit 1
done
