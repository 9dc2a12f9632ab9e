# round 5: hybrid walk phase stamps on the final tree (576-row walk)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05x
mkdir -p $OUT
RDN_WALK=1 timeout -k 10 300 python -u tools/hyb_stamps.py > $OUT/hyb_stamps_walk576.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/hyb_stamps_walk576.log; exit $rc
