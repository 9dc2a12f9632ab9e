# round 5: CBAM pointwise passes without per-row edge checks (rows outside [0, L) are zero by
# construction).  A/B (prev = last commit), stamps, GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05o
mkdir -p $OUT
for spec in ${SPECS:-ADSDN:10000:f16 APIDN:16384:f16 APIDN:10000:f16}; do
  IFS=: read -r a L dt <<< "$spec"
  RDN_ABLATE_L=$L ABLATE_ONLY=base,prev RDN_ABLATE_ARCH=$a timeout -k 10 300 python -u tools/ablate.py run $dt $dt > $OUT/ab_${a}_${L}_$dt.log 2>&1
  rc=$?; echo "$a L=$L"; grep -v amdgpu.ids $OUT/ab_${a}_${L}_$dt.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 200 python -u tools/team_stamps.py ADSDN f16 10000 stamps > $OUT/stamps_ADSDN.log 2>&1
rc=$?; grep -A10 "per phase" $OUT/stamps_ADSDN.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest_gpu.log | head -30; fi; exit $rc
