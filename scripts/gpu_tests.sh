# GPU test suite on one box (parity + diagnostics), output in gpurun_out/pytest_gpu.log
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 150 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | grep -v PASSED | head -40
grep -E "fp32 vs ref|passed|failed" gpurun_out/pytest_gpu.log | tail -5
exit $rc
