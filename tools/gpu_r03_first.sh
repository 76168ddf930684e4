set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_coverage.py -x -v -s --timeout 300 --timeout-method thread -k "auc or trainer_step" > gpurun_out/r03_auc.log 2>&1 &&
timeout -k 10 300 python -u bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-fp32 --no-cpu-baseline --steps 30 > gpurun_out/r03_c2.json 2> gpurun_out/r03_c2.err &&
timeout -k 10 400 python -u bench.py --rows-per-gpu 12500000 --no-fp32 --no-cpu-baseline --steps 30 > gpurun_out/r03_c5.json 2> gpurun_out/r03_c5.err
