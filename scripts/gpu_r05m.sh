# round 5: range tests against the fp32 noise floor at 2x
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05m
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_range_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_range.log 2>&1
rc=$?; tail -3 $OUT/pytest_range.log; if [ $rc -ne 0 ]; then grep -E "^E  |FAIL" $OUT/pytest_range.log | head -30; fi; exit $rc
