set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forward_gpu.py -x -v --timeout 120 --timeout-method thread -k "f16f8" > gpurun_out/pytest_f16f8.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "DSDN.*f16f8 max-abs|APIDN.*f16f8 max-abs|passed|failed|Error" gpurun_out/pytest_f16f8.log | head -16
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/throughput_table.py --archs ADSDN APIDN --dtypes f16f8 bf16x3 > gpurun_out/tp_cbam.log 2>&1
rc=$?; echo "tp rc=$rc"; grep "^|" gpurun_out/tp_cbam.log
