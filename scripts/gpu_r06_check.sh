# round 6: GPU suite + smoke, the 16-bit tolerance prints, the CBAM batch-1 path (latency split and a
# kernel trace: no aminmax kernel) -- one lease
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06d}
mkdir -p $OUT
STAGES="tests smoke" OUT=$OUT bash scripts/gpu.sh || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -q -s --timeout 150 --timeout-method thread \
  -k "test_16bit_within_tolerance or walk_saturation" > $OUT/tol.log 2>&1
rc=$?; tail -1 $OUT/tol.log; if [ $rc -ne 0 ]; then exit $rc; fi
for a in ADSDN APIDN RRCDNet; do
  B1_ARCH=$a timeout -k 10 300 python -u tools/batch1_profile.py > $OUT/batch1_$a.log 2>&1
  rc=$?; echo "$a: $(grep -m1 module $OUT/batch1_$a.log)"; if [ $rc -ne 0 ]; then tail -5 $OUT/batch1_$a.log; exit $rc; fi
done
B1_ARCH=ADSDN timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/b1kt -o kt -- python3 tools/batch1_profile.py > $OUT/b1kt.log 2>&1
rc=$?; echo "b1 trace rc=$rc"; exit $rc
