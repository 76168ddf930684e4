# where the overlapped untouched-row Adam starts: bench ms/step per setting
R=$GRAFT_REPO_ROOT
for st in step gather fwd; do
  FBN_ADAM_START=$st timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 40 > $R/gpurun_out/astart_$st.json 2>/dev/null || exit 1
  echo "$st $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/astart_$st.json)"
done
