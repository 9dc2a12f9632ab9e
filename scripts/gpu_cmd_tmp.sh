# scratch GPU command (changes per iteration)
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 8 > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-1800
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/throughput_table.py > gpurun_out/tp.log 2>&1
rc=$?; echo "tp rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
