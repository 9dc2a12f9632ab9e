# A/B of the CBAM f16 team kernel geometries (tools/geom_ab.py) + the CBAM GPU tests
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/geom
mkdir -p $OUT
timeout -k 10 300 python -u tools/geom_ab.py ${GEOM_ARGS} > $OUT/geom_ab.log 2>&1
rc=$?; echo "geom_ab rc=$rc"; grep -v amdgpu.ids $OUT/geom_ab.log | tail -5
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$GEOM_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "$GEOM_TESTS" > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
  exit $rc
fi
