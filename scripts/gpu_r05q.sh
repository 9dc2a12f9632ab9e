# round 5: ping-pong engine knobs (pf4, pf2, ld3) vs base, one process per network
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05q
mkdir -p $OUT
for spec in ${SPECS:-DenoiseCNN:10000:f16 RRCDNet:10000:f16-plain RRCDNet:10000:f16}; do
  IFS=: read -r a L dt <<< "$spec"
  RDN_ABLATE_L=$L ABLATE_ONLY=${ONLY:-base,pf4,pf2,ld3} RDN_ABLATE_ARCH=$a timeout -k 10 300 python -u tools/ablate.py run $dt $dt > $OUT/ab_${a}_${L}_$dt.log 2>&1
  rc=$?; echo "$a L=$L"; grep -v amdgpu.ids $OUT/ab_${a}_${L}_$dt.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
