# round 4, call 26: the committed final tree -- GPU suite, smoke, default bench line (a third lease)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_v.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu_v.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_v.log 2>&1
rc=$?; tail -1 $OUT/smoke_v.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > $OUT/bench_v.log 2>&1
rc=$?; tail -1 $OUT/bench_v.log | cut -c1-330; exit $rc
