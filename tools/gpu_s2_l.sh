# C2 with a shorter lazy window F (the window pass there is bound by its longest replay chain: lags up to F)
set -o pipefail
mkdir -p gpurun_out
C2="--dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-fp32"
for rnd in 1 2; do
  for F in 128 64 32; do
    timeout -k 10 200 python -u bench.py $C2 --lazy-window $F > gpurun_out/c2f_${F}_${rnd}.json 2> gpurun_out/c2f_${F}_${rnd}.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/c2f_${F}_${rnd}.json'));print('C2 F=$F rnd=$rnd', d['ms_per_step'], d['config']['hipgraph'])"
  done
done
