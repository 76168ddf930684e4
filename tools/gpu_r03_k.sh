# side-stream fork point A/B (claims / mmproj / gather / mlp0) x main-stream priority, two rounds
set -o pipefail
for rnd in 1 2; do
  for cfg in "X=0" "FBN_SIDE_AFTER_GATHER=1" "FBN_SIDE_AFTER_MMPROJ=1" "FBN_SIDE_AFTER_MLP0=1"; do
    for pr in "" "--main-priority"; do
      tag=$(echo "$cfg$pr" | tr -d ' =_-' | tr 'A-Z' 'a-z')
      env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 --probe-steps 0 $pr > gpurun_out/r03k_${tag}_$rnd.json 2> gpurun_out/r03k_${tag}_$rnd.err || exit 1
    done
  done
done
