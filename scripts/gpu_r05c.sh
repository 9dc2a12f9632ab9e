# round 5: RDN_F16MIX walk -- parity tests, A/B timing against the tiled hybrid, range / headline tests
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05c
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_forward_gpu.py -x -v --timeout 120 --timeout-method thread -k "walk" > $OUT/pytest_walk.log 2>&1
rc=$?; tail -3 $OUT/pytest_walk.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_walk.log | head -30; exit $rc; fi
timeout -k 10 300 python -u tools/walk_ab.py RRCDNet:f16 RRCDNet:f16-plain DenoiseCNN:f16 > $OUT/walk_ab.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/walk_ab.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_range_gpu.py tests/test_headline_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_range.log 2>&1
rc=$?; tail -3 $OUT/pytest_range.log; exit $rc
