# round 5: hybrid walk -- the corrected tail skips blocks beyond L + 8 on a spectrum's last tiles; A/B + walk tests
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05w
mkdir -p $OUT
for L in 10000 16384 3000; do
  RDN_WALK=1 RDN_ABLATE_L=$L ABLATE_ONLY=base,prev RDN_ABLATE_ARCH=RRCDNet timeout -k 10 300 python -u tools/ablate.py run f16 f16 > $OUT/ab_tailskip_$L.log 2>&1
  rc=$?; echo "L=$L"; grep -v amdgpu.ids $OUT/ab_tailskip_$L.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "walk or headline or RRCDNet or range" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "FAIL|^E " $OUT/pytest.log | head -20; fi; exit $rc
