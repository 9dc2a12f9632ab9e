# round 5 final evidence on the final tree, in ONE session: GPU suite, smoke, parity table, the default
# bench line, the rocprofv3 kernel trace of the same bench command (its kernel_stats CSVs are copied
# into profiles/r05 by tools/summarize_profiles.py), PMC passes (each its own process), throughput table
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/final
mkdir -p $OUT
STAGES=${STAGES:-tests smoke parity bench kt pmc throughput}
if [[ " $STAGES " == *" tests "* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -1 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest_gpu.log | head -20; exit $rc; fi
fi
if [[ " $STAGES " == *" smoke "* ]]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; tail -1 $OUT/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [[ " $STAGES " == *" parity "* ]]; then
  timeout -k 10 300 python -u tools/parity_report.py --out $OUT/parity.md > $OUT/parity.log 2>&1
  rc=$?; tail -2 $OUT/parity.md; if [ $rc -ne 0 ]; then exit $rc; fi
fi
INNER="$(echo "$STAGES" | tr ' ' '\n' | grep -x 'bench\|kt\|pmc' | tr '\n' ' ')"
if [ -n "$INNER" ]; then
  STAGES="$INNER" bash scripts/gpu_final.sh
  rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [[ " $STAGES " == *" throughput "* ]]; then
  timeout -k 10 400 python -u tools/throughput_table.py --out $OUT/throughput.md > $OUT/throughput.log 2>&1
  rc=$?; tail -3 $OUT/throughput.log; exit $rc
fi
