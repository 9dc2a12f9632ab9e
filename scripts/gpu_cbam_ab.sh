# CBAM f16 parity subset + A/B (tools/ablate.py variants) on ADSDN / APIDN.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "(ADSDN or APIDN) and (f16 or xcd) and not f16f8" > gpurun_out/pytest_cbam16.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/pytest_cbam16.log | head -10; tail -1 gpurun_out/pytest_cbam16.log
if [ $rc -ne 0 ]; then exit $rc; fi
for a in ADSDN APIDN; do
RDN_ABLATE_ARCH=$a timeout -k 10 300 python -u tools/ablate.py run f16 > gpurun_out/ablate_$a.log 2>&1
rc=$?; echo "ablate $a rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate_$a.log | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
done
