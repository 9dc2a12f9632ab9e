# scratch GPU command (changes per iteration)
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
: > gpurun_out/stamps.log
for v in stamps stamps_pre0 stamps_pre16; do
  for dt in bf16x3 bf16 fp32; do
    timeout -k 10 120 python -u tools/team_stamps.py APIDN $dt 10000 $v >> gpurun_out/stamps.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "stamps rc=$rc"; exit $rc; fi
  done
done
timeout -k 10 300 python -u tools/throughput_table.py > gpurun_out/tp.log 2>&1
rc=$?; echo "tp rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
