# round 6: headline batch-size sweep (the walk's last-round tail) + CBAM batch-1 after the fill merge
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06e}
mkdir -p $OUT
for B in 8192 16384 32768 8192; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --sustained-seconds 0 --no-variants --no-batch1 \
    --no-pipeline --batch $B > $OUT/bench_b$B.log 2>&1
  rc=$?; echo "B=$B $(tail -1 $OUT/bench_b$B.log | cut -c100-260)"; if [ $rc -ne 0 ]; then exit $rc; fi
done
for a in ADSDN APIDN; do
  B1_ARCH=$a timeout -k 10 300 python -u tools/batch1_profile.py > $OUT/batch1_$a.log 2>&1
  rc=$?; echo "$a: $(grep -m1 module $OUT/batch1_$a.log)"; if [ $rc -ne 0 ]; then tail -5 $OUT/batch1_$a.log; exit $rc; fi
done
