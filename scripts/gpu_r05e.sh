# round 5: diagnostic ablations of the walk kernels (wrong results: one component removed each)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05e
mkdir -p $OUT
export RDN_WALK=1
export ABLATE_ONLY=base,nobar,noaload,nolds,nomfma,nostore
RDN_ABLATE_ARCH=RRCDNet timeout -k 10 300 python -u tools/ablate.py run f16-plain f16 > $OUT/ablate_walk_diag.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_walk_diag.log; exit $rc
