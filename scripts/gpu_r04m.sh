# round 4, call 14: false range errors on 256-row edge tiles (smoke fell back to fp32 in call 13): status
# words of comb (before) vs track (rows outside [0, L) untracked) on the smoke inputs; f16-first MFMA order A/B; the regression test
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
timeout -k 10 120 python -u tools/dbg_short.py comb track > $OUT/dbg_short_m.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/dbg_short_m.log; if [ $rc -ne 0 ]; then exit $rc; fi
ABLATE_ONLY=track,f16first timeout -k 10 200 python -u tools/ablate.py run f16mix f16f8 > $OUT/ablate_m.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_m.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_range_gpu.py -m gpu -x -q -s --timeout 120 --timeout-method thread -k "false_range" > $OUT/pytest_range_m.log 2>&1
rc=$?; tail -3 $OUT/pytest_range_m.log; exit $rc
