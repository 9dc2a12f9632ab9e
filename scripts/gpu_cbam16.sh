# CBAM networks on the f16 ping-pong team kernel: parity subset, then throughput.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-(ADSDN or APIDN) and f16 and not f16f8}" > gpurun_out/pytest_cbam16.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/pytest_cbam16.log | head -20; tail -2 gpurun_out/pytest_cbam16.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for a in ADSDN APIDN; do
  timeout -k 10 200 python -u bench.py --arch $a --dtype f16 --batch 2048 --steps 5 --warmup 1 --no-cpu-baseline --no-variants --no-pipeline --no-batch1 > gpurun_out/bench_$a.log 2>&1
  rc2=$?; echo "bench $a rc=$rc2"; tail -1 gpurun_out/bench_$a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
  if [ $rc2 -ne 0 ]; then exit $rc2; fi
done
exit $rc
