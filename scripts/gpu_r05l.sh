# round 5: compensated fp32 in the CBAM kernels: chunk 6 (base) / 4 / 3 / 2 vs one plain chain (rescomp0):
# scaled-input error against float64 per input, over the reference's distance and over the fp32 noise
# floor (test_range_gpu's bar); then the range tests
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05l
mkdir -p $OUT
timeout -k 10 600 python -u tools/ablate.py scaled ${SCALED_ARCHS:-ADSDN APIDN DSDN DenoiseCNN RRCDNet PIDN} > $OUT/scaled3.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/scaled3.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_range_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_range.log 2>&1
rc=$?; tail -3 $OUT/pytest_range.log; if [ $rc -ne 0 ]; then grep -E "^E  |FAIL" $OUT/pytest_range.log | head -30; fi; exit $rc
