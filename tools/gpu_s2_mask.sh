# side stream on a CU subset (FBN_SIDE_CU_MASK; the stream is made at trainer init, so separate bench
# runs, interleaved): all CUs vs 3 of 4 vs 1 of 2
set -o pipefail
mkdir -p gpurun_out
for rnd in 1 2; do
  for M in all 77777777 55555555; do
    if [ $M = all ]; then E=""; else E="FBN_SIDE_CU_MASK=$M"; fi
    env $E timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 > gpurun_out/mask_${M}_${rnd}.json 2> gpurun_out/mask_${M}_${rnd}.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/mask_${M}_${rnd}.json'));print('mask=$M rnd=$rnd', d['ms_per_step'], d['config']['hipgraph'])"
  done
done
