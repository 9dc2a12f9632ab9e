# round 5: B-prefetch depth / load spacing of the walk kernels (A/B in one process)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05i
mkdir -p $OUT
export RDN_WALK=1 ABLATE_ONLY=base,pf2,pf4,ld3
RDN_ABLATE_ARCH=RRCDNet timeout -k 10 300 python -u tools/ablate.py run f16-plain f16 > $OUT/ablate_pf.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_pf.log; exit $rc
