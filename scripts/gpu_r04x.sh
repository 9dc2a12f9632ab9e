# round 4, call 28: corrected-product MFMA interleave only on the non-residual convs (resplain = this
# tree, cur = the committed one): DSDN f16f8 (residual) and the hybrid; then the whole GPU suite + smoke
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
RDN_ABLATE_ARCH=DSDN ABLATE_ONLY=cur,resplain timeout -k 10 200 python -u tools/ablate.py run f16f8 > $OUT/ablate_x_dsdn.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_x_dsdn.log; if [ $rc -ne 0 ]; then exit $rc; fi
ABLATE_ONLY=cur,resplain timeout -k 10 200 python -u tools/ablate.py run f16mix > $OUT/ablate_x.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_x.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_x.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu_x.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_x.log 2>&1
rc=$?; tail -1 $OUT/smoke_x.log; exit $rc
