# A/B of a host-side env knob (tools/env_ab.py) + the CBAM f16 GPU tests; ENV_AB_ARGS passes --var/--value
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/env_ab
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "(ADSDN or APIDN) and (f16 or xcd) and not f16f8" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $OUT/pytest.log | head -10; exit $rc; fi
timeout -k 10 300 python -u tools/env_ab.py ${ENV_AB_ARGS} > $OUT/env_ab.log 2>&1
rc=$?; echo "env_ab rc=$rc"; grep -v amdgpu.ids $OUT/env_ab.log | tail -5
exit $rc
