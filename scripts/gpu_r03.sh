# Round-3 GPU check: the new/changed parity tests first (fail fast), then the whole -m gpu suite,
# smoke(), and the default bench line (with the configs 2/4/5 keys).  Every GPU step has its own
# time limit; the script stops at the first step that fails hard.
#   STAGES="new all smoke bench" bash scripts/gpu_r03.sh
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
stages=${STAGES:-new all smoke bench}
hard() { [ $1 -ne 0 ] && [ $1 -ne 1 ]; }
for st in $stages; do
  case $st in
    new)
      timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 200 --timeout-method thread -m gpu \
        tests/test_headline_gpu.py tests/test_pipeline_gpu.py tests/test_generator_gpu.py tests/test_evaluate_gpu.py \
        tests/test_bench_multirank_gpu.py > gpurun_out/pytest_new.log 2>&1
      rc=$?; echo "pytest new rc=$rc"; grep -E "PASSED|FAILED|ERROR|Error|assert|heldout|max-abs" gpurun_out/pytest_new.log | grep -v "^tests.*PASSED" | tail -30; tail -2 gpurun_out/pytest_new.log
      if hard $rc; then exit $rc; fi ;;
    all)
      timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/pytest_all.log 2>&1
      rc=$?; echo "pytest all rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_all.log | head -20; tail -2 gpurun_out/pytest_all.log
      if hard $rc; then exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
      if [ $rc -ne 0 ]; then exit $rc; fi ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-3000
      if [ $rc -ne 0 ]; then exit $rc; fi ;;
    config1)
      for spec in "DenoiseCNN fp32" "RRCDNet f16" "RRCDNet fp32"; do
        set -- $spec
        timeout -k 10 600 python -u tools/config1_eval.py --n 1000 --cpu-n ${CPU_N:-300} --arch $1 --dtype $2 \
          --out gpurun_out/r03/config1_$1_$2.json > gpurun_out/config1_$1_$2.log 2>&1
        rc=$?; echo "config1 $1 $2 rc=$rc"; grep -E "max_|spectra_per_s" gpurun_out/r03/config1_$1_$2.json
        if [ $rc -ne 0 ]; then exit $rc; fi
      done ;;
    config4)
      timeout -k 10 900 python -u tools/config4.py --total ${C4_TOTAL:-12500000} --out gpurun_out/r03/config4_shard.json \
        > gpurun_out/config4.log 2>&1
      rc=$?; echo "config4 rc=$rc"; tail -1 gpurun_out/config4.log | cut -c1-2000
      if [ $rc -ne 0 ]; then exit $rc; fi ;;
  esac
done
exit 0
