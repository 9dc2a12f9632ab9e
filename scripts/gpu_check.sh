# GPU round check: parity tests, then short benches for each engine dtype, then a kernel-trace profile.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for dt in bf16 bf16x3 fp32; do
  B=8192; [ $dt = fp32 ] && B=1024; [ $dt = bf16x3 ] && B=2048
  timeout -k 10 200 python -u bench.py --dtype $dt --batch $B --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$dt.log 2>&1
  rc=$?; echo "bench $dt rc=$rc"; tail -1 gpurun_out/bench_$dt.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
done
