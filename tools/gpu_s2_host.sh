# host enqueue time per eager step (GPU held behind a sleep): side stream vs serial side passes, C3 and C2
set -o pipefail
mkdir -p gpurun_out
for S in 0 1; do
  FBN_SIDE_SERIAL=$S HP_NOPROF=1 timeout -k 10 200 python -u tools/host_profile.py 2>&1 | grep -v amdgpu.ids | sed "s/^/C3 serial=$S: /" || exit 1
  FBN_SIDE_SERIAL=$S HP_NOPROF=1 EG_D=16 EG_V=1000000 EG_B=4096 timeout -k 10 200 python -u tools/host_profile.py 2>&1 | grep -v amdgpu.ids | sed "s/^/C2 serial=$S: /" || exit 1
done
