set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_full.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_profile.sh
rc=$?; echo "profile rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/throughput_table.py > gpurun_out/tp.log 2>&1
rc=$?; echo "tp rc=$rc"
