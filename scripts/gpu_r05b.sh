# round 5: walk variants A/B (prev = the first walk commit, base = carry ops interleaved, w512 = 512-row walk tiles)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05b
mkdir -p $OUT
export RDN_WALK=1
RDN_ABLATE_ARCH=DenoiseCNN timeout -k 10 300 python -u tools/ablate.py run f16 > $OUT/ablate_dcnn.log 2>&1
rc=$?; cat $OUT/ablate_dcnn.log | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
RDN_ABLATE_ARCH=RRCDNet timeout -k 10 300 python -u tools/ablate.py run f16-plain > $OUT/ablate_rrcd.log 2>&1
rc=$?; cat $OUT/ablate_rrcd.log | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
unset RDN_WALK
timeout -k 10 300 python -u tools/walk_ab.py > $OUT/walk_ab.log 2>&1
rc=$?; cat $OUT/walk_ab.log | grep -v amdgpu.ids; exit $rc
