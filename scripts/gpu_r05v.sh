# round 5: a third lease on the final tree -- the default bench line, then a 60-s sustained window
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05v
mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; tail -1 $OUT/bench.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi
grep "^{" $OUT/bench.log | tail -1 > $OUT/bench.json
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-configs --no-variants --no-pipeline --no-batch1 --sustained-seconds 60 --sustained-spectra 8000000 > $OUT/bench_sustained60.log 2>&1
rc=$?; tail -1 $OUT/bench_sustained60.log | cut -c1-300; grep "^{" $OUT/bench_sustained60.log | tail -1 > $OUT/bench_sustained60.json; exit $rc
