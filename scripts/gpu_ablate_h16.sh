# Ping-pong engine knobs (tools/ablate.py variants built in the container), timed interleaved in one
# process on RRCDNet (f16-plain and the 'f16' hybrid) and DenoiseCNN (f16).
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
for a in ${ABLATE_ARCHS:-RRCDNet DenoiseCNN}; do
  RDN_ABLATE_ARCH=$a timeout -k 10 300 python -u tools/ablate.py run ${ABLATE_DTYPES:-f16-plain f16} > gpurun_out/r03/ablate_h16_$a.log 2>&1
  rc=$?; echo "ablate $a rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/ablate_h16_$a.log | tail -12
  if [ $rc -ne 0 ]; then exit $rc; fi
done
