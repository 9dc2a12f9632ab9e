# round 4, call 24: the tree after removing this round's diagnostic-only knobs (compiled out before):
# GPU suite, smoke, a short bench line
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_t.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu_t.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_t.log 2>&1
rc=$?; tail -1 $OUT/smoke_t.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs > $OUT/bench_t.log 2>&1
rc=$?; tail -1 $OUT/bench_t.log | cut -c1-330; exit $rc
