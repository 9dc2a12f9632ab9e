# Round-3 batch C: GPU suite on the working tree (edge-tile post-pass), the RDN_F16MIX tail sweep on
# config 1's 1000 spectra, throughput A/B (edge post-pass vs masked epilogues; tails 3/4/5), CBAM A/B
# and per-tile stamps.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "pytest all rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_all.log | head -20; tail -1 gpurun_out/pytest_all.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/f16mix_tail_eval.py base tail4 tail5 > gpurun_out/r03/f16mix_tail_eval.log 2>&1
rc=$?; echo "tail eval rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/f16mix_tail_eval.log
if [ $rc -ne 0 ]; then exit $rc; fi
ABLATE_ONLY=base,edgesel,tail4,tail5 ABLATE_ARCHS="RRCDNet" ABLATE_DTYPES="f16 f16-plain" bash scripts/gpu_ablate_h16.sh || exit 1
ABLATE_ONLY=base,edgesel ABLATE_ARCHS="DenoiseCNN PIDN" ABLATE_DTYPES="f16" bash scripts/gpu_ablate_h16.sh || exit 1
for a in ADSDN APIDN; do
  ABLATE_ONLY=base,edgesel RDN_ABLATE_ARCH=$a timeout -k 10 300 python -u tools/ablate.py run f16 > gpurun_out/r03/ablate_edge_$a.log 2>&1
  rc=$?; echo "ablate $a rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/ablate_edge_$a.log | tail -2
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 120 python -u tools/team_stamps.py ADSDN f16 10000 stamps > gpurun_out/r03/stamps16_tiles_post_ADSDN.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -E "tile  0|tile  1:|tile 15|spectra/s" gpurun_out/r03/stamps16_tiles_post_ADSDN.log
