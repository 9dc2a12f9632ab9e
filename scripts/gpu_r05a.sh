# round 5: walk geometry -- parity tests, then the A/B timing against the 640-row tiles; status word
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_forward_gpu.py -x -v --timeout 120 --timeout-method thread -k "walk" > $OUT/pytest_walk.log 2>&1
rc=$?; tail -3 $OUT/pytest_walk.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_walk.log | head -20; exit $rc; fi
timeout -k 10 300 python -u tools/walk_ab.py > $OUT/walk_ab.log 2>&1
rc=$?; cat $OUT/walk_ab.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests/test_range_gpu.py tests/test_evaluate_gpu.py tests/test_headline_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_range.log 2>&1
rc=$?; tail -3 $OUT/pytest_range.log; exit $rc
