cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
FBN_SERIAL_ADAM=1 timeout -k 10 300 python $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_serial.json 2>&1 && \
FBN_SERIAL_ADAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_serial -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_serial.log 2>&1
