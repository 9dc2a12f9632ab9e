set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_evaluate_gpu.py -q -s --timeout 200 --timeout-method thread > gpurun_out/pytest_eval.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_eval.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/config1_eval.py --n 1000 --cpu-n 300 --out gpurun_out/config1.json > gpurun_out/config1.log 2>&1
rc2=$?; echo "config1 rc=$rc2"; tail -30 gpurun_out/config1.log
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc3=$?; echo "bench rc=$rc3"; tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], json.dumps(d['batch1']), json.dumps(d['cpu_baseline']))"
exit $rc
