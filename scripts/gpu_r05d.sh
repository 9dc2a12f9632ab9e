# round 5: phase stamps of the RDN_F16MIX walk and of the tiled hybrid (same build)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05d
mkdir -p $OUT
RDN_WALK=1 timeout -k 10 200 python -u tools/hyb_stamps.py > $OUT/stamps_walk.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/stamps_walk.log; if [ $rc -ne 0 ]; then exit $rc; fi
RDN_WALK=0 timeout -k 10 200 python -u tools/hyb_stamps.py > $OUT/stamps_tiles.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/stamps_tiles.log; exit $rc
