# round 4, call 19: CBAM hand-off waits bounded by the wall clock (s_memrealtime, 0.3 s): the timeout
# test with its measured latency, the CBAM tests, and the team kernels' speed
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_forward_gpu.py -m gpu -q -s --timeout 120 --timeout-method thread -k "cbam" > $OUT/pytest_cbam_p.log 2>&1
rc=$?; grep -E "timeout reported|passed|failed|FAILED" $OUT/pytest_cbam_p.log | tail -8; if [ $rc -ne 0 ]; then exit $rc; fi
for a in ADSDN APIDN; do
  timeout -k 10 200 python -u bench.py --arch $a --dtype f16 --batch 2048 --steps 10 --warmup 2 --no-cpu-baseline --no-variants --no-pipeline --no-batch1 --no-configs > $OUT/bench_$a.log 2>&1
  rc=$?; tail -1 $OUT/bench_$a.log | cut -c1-260; if [ $rc -ne 0 ]; then exit $rc; fi
done
