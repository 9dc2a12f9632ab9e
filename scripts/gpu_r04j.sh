# round 4, call 11: tail operands issued before the staged planes are written, LDS-only barrier (stg = this tree)
# finer phase stamps (10 phases)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
ABLATE_ONLY=lbar,stg timeout -k 10 200 python -u tools/ablate.py run f16mix > $OUT/ablate_j.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_j.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/hyb_stamps.py > $OUT/hyb_stamps_j.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/hyb_stamps_j.log; exit $rc
