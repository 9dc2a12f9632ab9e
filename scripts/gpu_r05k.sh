# round 5: A/B of a hybrid-walk change (prev = last commit) on the walk
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05k
mkdir -p $OUT
RDN_WALK=1 ABLATE_ONLY=base,prev RDN_ABLATE_ARCH=RRCDNet timeout -k 10 300 python -u tools/ablate.py run f16 f16 > $OUT/ablate.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate.log; exit $rc
