# round 4, call 27: the range regression test with its exact exception type
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_range_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "false_range or saturation" > gpurun_out/r04/pytest_w.log 2>&1
rc=$?; tail -1 gpurun_out/r04/pytest_w.log; exit $rc
