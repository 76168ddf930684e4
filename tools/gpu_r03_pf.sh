# two-pass table-Adam prefetch: bit-identity tests, then C3 bench A/B (one-pass vs two-pass)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -v --timeout 200 --timeout-method thread -k "prefetch or lazy or window or deferred or owner" > gpurun_out/r03_pf_tests.log 2>&1 &&
FBN_PREFETCH_ONEPASS=1 timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_pf_one.json 2> gpurun_out/r03_pf_one.err &&
timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_pf_two.json 2> gpurun_out/r03_pf_two.err &&
FBN_PREFETCH_ONEPASS=1 timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_pf_one2.json 2> gpurun_out/r03_pf_one2.err &&
timeout -k 10 300 python -u bench.py --no-fp32 --no-cpu-baseline --steps 40 > gpurun_out/r03_pf_two2.json 2> gpurun_out/r03_pf_two2.err
