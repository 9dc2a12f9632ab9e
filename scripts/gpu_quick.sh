# GPU: parity tests (subset via PYTEST_K), then a short bench line.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 150 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"
grep -E "FAILED|ERROR|Error" gpurun_out/pytest_gpu.log | head -30
tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -1 gpurun_out/bench.log | cut -c1-2500
exit $rc
