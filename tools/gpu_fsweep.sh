# Lazy window F sweep: separate bench runs, interleaved (the ring is sized by F, so no in-process A/B)
set -o pipefail
mkdir -p gpurun_out
for rnd in 1 2; do
  for F in 128 256 512; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 --lazy-window $F $EXTRA > gpurun_out/fs_${F}_${rnd}.json 2> gpurun_out/fs_${F}_${rnd}.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/fs_${F}_${rnd}.json'));print('F=$F rnd=$rnd', d['ms_per_step'])"
  done
done
