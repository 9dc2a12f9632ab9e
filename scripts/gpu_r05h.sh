# round 5: batch-1 call breakdown + the module-path tests
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_forward_gpu.py tests/test_range_gpu.py tests/test_evaluate_gpu.py -x -q --timeout 120 --timeout-method thread -k "speculative or packing or range or module or evaluate or batch" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest.log | head; exit $rc; fi
timeout -k 10 300 python -u tools/batch1_profile.py > $OUT/batch1.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/batch1.log | head -30; exit $rc
