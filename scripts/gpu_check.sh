set +e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o r1 -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
echo "prof rc=$?"
