# round 5: CBAM MODE_H8 team taint (a saturated tile NaNs its whole spectrum); range + CBAM tests
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05s
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -k "${PYTEST_K:-range or cbam or CBAM or ADSDN or APIDN}" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; grep -E "saturated|finite fraction" $OUT/pytest.log | head -20; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|^E " $OUT/pytest.log | head -30; fi; exit $rc
