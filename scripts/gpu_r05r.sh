# round 5: config 4 at its stated scale per rank -- 100 M spectra over 8 GPUs is 12.5 M per rank; rank 0
# of that run owns indices [0, 12.5 M), which this one-GPU run processes (W = 1, --total 12,500,000),
# each network its own process (<= 140 s each); plus the range tests (denormal flush)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05r
mkdir -p $OUT
for a in RRCDNet DSDN ADSDN; do
  timeout -k 10 400 python -u tools/config4.py --total 12500000 --archs $a --out $OUT/config4_12p5M_$a.json > $OUT/config4_$a.log 2>&1
  rc=$?; echo "$a rc=$rc"; tail -1 $OUT/config4_$a.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 600 python -u -m pytest tests/test_range_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_range.log 2>&1
rc=$?; tail -2 $OUT/pytest_range.log; exit $rc
