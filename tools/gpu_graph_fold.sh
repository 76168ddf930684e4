set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trainer.py -k "interleave or prefetch" > gpurun_out/s2q_tests.log 2>&1 || exit 1
for FX in auto 1; do
  FBN_FIXUP_ON_SIDE=$FX timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32 --mode graph > gpurun_out/s2q_g_$FX.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/s2q_g_$FX.json'));print('graph fixup=$FX', d['ms_per_step'])"
done
