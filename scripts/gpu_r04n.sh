# round 4, call 15: the GPU suite with fp32-rerun warnings as failures, smoke, and the default bench line
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread > $OUT/pytest_gpu_n.log 2>&1
rc=$?; grep -E "heldout|config 1|passed|failed|Error|FAILED" $OUT/pytest_gpu_n.log | tail -20
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_n.log 2>&1
rc2=$?; tail -1 $OUT/smoke_n.log; if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 600 python -u bench.py > $OUT/bench_n.log 2>&1
rc3=$?; tail -1 $OUT/bench_n.log | cut -c1-600; exit $(( rc | rc3 ))
