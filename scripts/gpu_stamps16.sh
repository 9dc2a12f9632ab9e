set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "(ADSDN or APIDN) and xcd" > gpurun_out/pytest_cbam16.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/pytest_cbam16.log | head -10; tail -1 gpurun_out/pytest_cbam16.log
if [ $rc -ne 0 ]; then exit $rc; fi
for a in ADSDN APIDN; do
timeout -k 10 120 python -u tools/team_stamps.py $a f16 10000 stamps > gpurun_out/stamps16_$a.log 2>&1
rc=$?; echo "stamps $a rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps16_$a.log | tail -17 | grep -v " 0.000e+00 (  0.0%)"
if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
rc=$?; echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate.log | tail -3
