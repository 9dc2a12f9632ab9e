# 16-bit GPU tests + A/B of the ping-pong stem (tools/ablate.py base vs stem1 = the item loop)
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/stem_ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "f16 and not f16f8" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $OUT/pytest.log | head -10; exit $rc; fi
for a in RRCDNet DenoiseCNN PIDN ADSDN; do
RDN_ABLATE_ARCH=$a ABLATE_ONLY=${ABL:-base,stem1} timeout -k 10 300 python -u tools/ablate.py run f16 f16-plain > $OUT/ablate_$a.log 2>&1
rc=$?; echo "ablate $a rc=$rc"; grep -v amdgpu.ids $OUT/ablate_$a.log | grep "ms" | tail -6
if [ $rc -ne 0 ]; then exit $rc; fi
done
