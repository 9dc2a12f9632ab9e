# round 4, call 10: LDS-only barrier before the left stem (lbar = this tree, mhead = call 9's), and the
# finer phase stamps (10 phases)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
ABLATE_ONLY=mhead,lbar timeout -k 10 200 python -u tools/ablate.py run f16mix > $OUT/ablate_i.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_i.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/hyb_stamps.py > $OUT/hyb_stamps_i.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/hyb_stamps_i.log; exit $rc
