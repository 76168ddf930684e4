# side-stream passes in sequence on the main stream (FBN_SIDE_SERIAL=1: no cross-queue edges in a
# replayed graph) vs on the side stream: C2 (graph-replayed) and C3 --mode graph, interleaved bench runs
set -o pipefail
mkdir -p gpurun_out
C2="--dim 16 --batch 4096 --rows-per-gpu 1000000"
for rnd in 1 2; do
  for S in 0 1; do
    FBN_SIDE_SERIAL=$S timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 $C2 > gpurun_out/ser_c2_${S}_${rnd}.json 2> gpurun_out/ser_c2_${S}_${rnd}.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ser_c2_${S}_${rnd}.json'));print('C2 serial=$S rnd=$rnd', d['ms_per_step'], d['config']['hipgraph'], d['config'].get('launch_mode_trial_ms_per_step'))"
    FBN_SIDE_SERIAL=$S timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 --mode graph > gpurun_out/ser_c3g_${S}_${rnd}.json 2> gpurun_out/ser_c3g_${S}_${rnd}.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ser_c3g_${S}_${rnd}.json'));print('C3 graph serial=$S rnd=$rnd', d['ms_per_step'])"
  done
done
