# round 4, call 29: the unfused PyTorch-ROCm eager baseline re-measured (fp32 and bf16; VERDICT r03
# weak 10: it dated from round 1), with one FETCH_SIZE / WRITE_SIZE pass each for the fp32 path
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r04/unfused
mkdir -p $OUT
for dt in fp32 bf16; do
  timeout -k 10 300 python -u tools/unfused_baseline.py --dtype $dt --out $OUT/unfused_$dt.json > $OUT/unfused_$dt.log 2>&1
  rc=$?; tail -1 $OUT/unfused_$dt.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/pmc_$ctr -o p -- python3 tools/unfused_baseline.py --dtype fp32 --steps 2 > $OUT/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/pmc_$ctr.log; exit $rc; fi
done
