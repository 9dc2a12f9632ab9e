# Round validation on one MI355X: GPU parity suite, smoke(), default bench line, unfused baseline.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/unf
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-600
if [ $rc -ne 0 ]; then exit $rc; fi
for dt in fp32 bf16; do
  timeout -k 10 240 python -u tools/unfused_baseline.py --dtype $dt --out gpurun_out/unf/unfused_$dt.json > gpurun_out/unf/unfused_$dt.log 2>&1
  rc=$?; echo "unfused $dt rc=$rc"; tail -1 gpurun_out/unf/unfused_$dt.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/unf/pmc_${dt}_$ctr -o p -- python3 tools/unfused_baseline.py --dtype $dt --steps 2 --warmup 2 --batch 64 > gpurun_out/unf/pmc_${dt}_$ctr.log 2>&1
    rc=$?; echo "pmc unfused $dt $ctr rc=$rc"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/unf/pmc_${dt}_$ctr.log; exit $rc; fi
  done
done
