# round 5: walk occupancy experiment (12 waves per CU, RDN_WALK_WAVES=12, spills) vs base
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05u
mkdir -p $OUT
for spec in DenoiseCNN:f16 RRCDNet:f16-plain; do
  IFS=: read -r a dt <<< "$spec"
  RDN_WALK=1 ABLATE_ONLY=${ONLY:-base,w12} RDN_ABLATE_ARCH=$a timeout -k 10 300 python -u tools/ablate.py run $dt $dt > $OUT/ab_w12_$a.log 2>&1
  rc=$?; echo "$a"; grep -v amdgpu.ids $OUT/ab_w12_$a.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
