# round 5: A/B of a ping-pong engine variant (VARIANT vs base) on the walk networks and the CBAM teams
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05p
mkdir -p $OUT
V=${VARIANT:-estag}
for spec in ${SPECS:-DenoiseCNN:10000:f16 RRCDNet:10000:f16-plain RRCDNet:10000:f16 PIDN:10000:f16 DSDN:10000:f16 ADSDN:10000:f16}; do
  IFS=: read -r a L dt <<< "$spec"
  RDN_ABLATE_L=$L ABLATE_ONLY=base,$V RDN_ABLATE_ARCH=$a timeout -k 10 300 python -u tools/ablate.py run $dt $dt > $OUT/ab_${V}_${a}_${L}_$dt.log 2>&1
  rc=$?; echo "$a L=$L"; grep -v amdgpu.ids $OUT/ab_${V}_${a}_${L}_$dt.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
