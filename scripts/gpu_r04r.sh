# round 4, call 22: bench.py --gpus 2 without a launcher (its own two ranks, gloo on the box's GPU), and
# the other multi-rank tests
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_bench_multirank_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread > $OUT/pytest_multirank_r.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest_multirank_r.log | tail -6; exit $rc
