# Round-3 batch: GPU test suite on the working tree, ping-pong engine A/B (EDGE branch, priorities),
# CBAM A/B + per-tile stamps, then the evidence stages.  Stops at the first hard failure.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "pytest all rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_all.log | head -20; tail -1 gpurun_out/pytest_all.log
if [ $rc -ne 0 ]; then exit $rc; fi
ABLATE_ONLY=base,edgesel,hprio1,hprio2 ABLATE_ARCHS="RRCDNet DenoiseCNN" bash scripts/gpu_ablate_h16.sh || exit 1
for a in ADSDN APIDN; do
  ABLATE_ONLY=base,edgesel RDN_ABLATE_ARCH=$a timeout -k 10 300 python -u tools/ablate.py run f16 > gpurun_out/r03/ablate_edge_$a.log 2>&1
  rc=$?; echo "ablate $a rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/ablate_edge_$a.log | tail -2
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 120 python -u tools/team_stamps.py $a f16 10000 stamps > gpurun_out/r03/stamps16_tiles_$a.log 2>&1
  rc=$?; echo "stamps $a rc=$rc"; grep -E "tile|spectra/s" gpurun_out/r03/stamps16_tiles_$a.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
STAGES="${EVIDENCE:-parity config1 throughput}" bash scripts/gpu_evidence.sh
