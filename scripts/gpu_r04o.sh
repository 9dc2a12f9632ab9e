# round 4, call 16: idle waves of short edge tiles zero their rows (stale LDS reached the 256-row
# hybrid's tracked halo rows through the wrapped taps); the false-range diagnostic, the range and
# headline tests, the whole GPU suite; interleaved corrected-product MFMAs A/B (ilv vs trk2)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
timeout -k 10 180 python -u tools/dbg_range.py f16 > $OUT/dbg_range_o.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/dbg_range_o.log | tail -8; if [ $rc -ne 0 ]; then exit $rc; fi
ABLATE_ONLY=trk2,ilv timeout -k 10 200 python -u tools/ablate.py run f16mix f16f8 > $OUT/ablate_o.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_o.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread > $OUT/pytest_gpu_o.log 2>&1
rc=$?; grep -E "config 1|passed|failed|FAILED" $OUT/pytest_gpu_o.log | tail -12; exit $rc
