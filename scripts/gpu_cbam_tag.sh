# CBAM f16 team kernel, tagged hand-off (RDN_T16_TAGGED): parity subset (incl. the forced-miss
# timeout tests), per-phase stamps tagged vs untagged, then the A/B timing in one process.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "(ADSDN or APIDN) and f16 and not f16f8" > gpurun_out/pytest_cbam16.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/pytest_cbam16.log | head -10; tail -1 gpurun_out/pytest_cbam16.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in stamps untag_stamps; do
for a in ADSDN APIDN; do
timeout -k 10 120 python -u tools/team_stamps.py $a f16 10000 $v > gpurun_out/r03/stamps16_${a}_$v.log 2>&1
rc=$?; echo "stamps $a $v rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/stamps16_${a}_$v.log | tail -17 | grep -v " 0.000e+00 (  0.0%)"
if [ $rc -ne 0 ]; then exit $rc; fi
done
done
for a in ADSDN APIDN; do
ABLATE_ONLY=${ABLATE_ONLY:-base,untag,saglobal,untag_saglobal,sleep2} RDN_ABLATE_ARCH=$a timeout -k 10 300 python -u tools/ablate.py run f16 > gpurun_out/r03/ablate_$a.log 2>&1
rc=$?; echo "ablate $a rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/ablate_$a.log | tail -4
if [ $rc -ne 0 ]; then exit $rc; fi
done
