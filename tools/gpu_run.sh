#!/bin/bash
# One GPU call, several steps, each under its own time limit; stops at the first failure.
# Usage (via gpurun): bash tools/gpu_run.sh <tag> <step> [<step> ...]
#   tests      the whole -m gpu suite (log: gpurun_out/<tag>/tests.log)
#   smoke      __graft_entry__.smoke()
#   bisect     the training-run AUC bisection (tests/parity_bisect.py): launcher runs with the
#              deterministic fold, the atomic fold (twice) and the IEEE-Adam library, then the
#              oracle ensemble report (gpurun_out/<tag>/auc_bisect.json)
#   step1      the first training step per tensor, HIP vs the float64 / fp32 oracle (parity_bisect step1)
#   bench      the default bench line (gpurun_out/<tag>/bench.json)
#   benchq     the bench without the CPU / fp32 / inference legs
#   zipf       the Zipf(1.05) bench line
#   c2         the C2 bench line (d 16, B 4096, 1 M rows)
#   shard      the sharded step as a one-rank RCCL job (per-GPU BatchNorm)
#   gather     the gather arms (tools/time_fields.py) at C3 and C2 shapes
#   gabl       the gather's ablations (FBN_FIELDS_ABL: no history loads / no stores / no other loads)
#   prof       rocprofv3 kernel trace + stats of the quick bench
#   pmc        the PMC passes (tools/gpu_pmc.sh)
#   ab:R:ARM1|ARM2|...   interleaved bench arms (tools/ab_arms.sh; an arm is "VAR=x VAR2=y", "-" = default)
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export PYTHONUNBUFFERED=1
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
             > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
           tail -3 $O/smoke.log ;;
    bisect)
      rc=0
      for arm in det:: nondet1:--nondet: nondet2:--nondet: ieee::tools/variants/libfibinet_hip_ieee.so; do
        IFS=: read -r t flag lib <<< "$arm"
        FBN_LIB_PATH=$lib timeout -k 10 300 python -m tests.parity_bisect hip --tag $t $flag --out $O/hip_$t.npz \
          >> $O/bisect.log 2>&1 || { rc=$?; break; }
      done
      if [ $rc -eq 0 ]; then
        timeout -k 10 600 python -m tests.parity_bisect report \
          --hip $O/hip_det.npz,$O/hip_nondet1.npz,$O/hip_nondet2.npz,$O/hip_ieee.npz --out $O/auc_bisect.json \
          >> $O/bisect.log 2>&1; rc=$?
      fi
      grep -E "^(hip|f64|fp32)" $O/bisect.log || true ;;
    step1) timeout -k 10 300 python -m tests.parity_bisect step1 --out $O/step1.json > $O/step1.log 2>&1; rc=$?
           tail -5 $O/step1.log ;;
    bench) timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json | head -c 600; echo ;;
    benchq) timeout -k 10 400 python bench.py --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 \
              > $O/benchq.json 2> $O/benchq.err; rc=$?; head -c 400 $O/benchq.json; echo ;;
    zipf) timeout -k 10 400 python bench.py --zipf 1.05 --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 \
            > $O/zipf.json 2> $O/zipf.err; rc=$?; head -c 400 $O/zipf.json; echo ;;
    c2) timeout -k 10 400 python bench.py --dim 16 --batch 4096 --rows-per-gpu 1000000 --no-cpu-baseline --no-cpu-plan \
          --no-inference --no-fp32 > $O/c2.json 2> $O/c2.err; rc=$?; head -c 400 $O/c2.json; echo ;;
    shard) FBN_BENCH_SHARD=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 \
             timeout -k 10 300 python bench.py --gpus 1 --no-fp32 --no-cpu-baseline --no-cpu-plan --no-inference \
             --bn local > $O/shard.json 2> $O/shard.err; rc=$?; head -c 400 $O/shard.json; echo ;;
    gather) { timeout -k 10 300 python tools/time_fields.py "plain5:" "plain10:FBN_FIELDS_HCH=10" \
                "plain20:FBN_FIELDS_HCH=20" "cmp5:FBN_FIELDS_CMP=1" "cmp8:FBN_FIELDS_CMP=1,FBN_FIELDS_HCH=8" \
                "cmp10:FBN_FIELDS_CMP=1,FBN_FIELDS_HCH=10" && \
              D=16 B=4096 V=1000000 timeout -k 10 300 python tools/time_fields.py "plain5:" "cmp5:FBN_FIELDS_CMP=1" \
                "cmp10:FBN_FIELDS_CMP=1,FBN_FIELDS_HCH=10"; } \
              > $O/gather.txt 2>&1; rc=$?; cat $O/gather.txt | grep -v Warn ;;
    gabl) timeout -k 10 300 python tools/time_fields.py "real:" "nohist:FBN_FIELDS_ABL=1" "nostore:FBN_FIELDS_ABL=2" \
            "noitem:FBN_FIELDS_ABL=4" "stores_only:FBN_FIELDS_ABL=5" "hist_only:FBN_FIELDS_ABL=6" "none:FBN_FIELDS_ABL=7" \
            > $O/gabl.txt 2>&1; rc=$?; grep -v Warn $O/gabl.txt ;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $O/prof -o run -- python $R/bench.py --no-cpu-baseline --no-cpu-plan --no-inference --no-fp32 \
             > $O/prof.log 2>&1); rc=$?; [ -f $O/prof/run_kernel_trace.csv ] && gzip -f $O/prof/run_kernel_trace.csv ;;
    pmc) bash tools/gpu_pmc.sh $TAG > $O/pmc.txt 2>&1; rc=$?; tail -40 $O/pmc.txt ;;
    ab:*) IFS=: read -r _ nr arms <<< "$step"; IFS='|' read -ra A <<< "$arms"
          for i in "${!A[@]}"; do [ "${A[$i]}" = "-" ] && A[$i]=""; done
          timeout -k 10 1100 bash tools/ab_arms.sh $nr "${A[@]}" > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "== $step rc=$rc $(date +%T)"
  [ $rc -eq 0 ] || exit $rc
done
