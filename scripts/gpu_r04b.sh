# round 4, call 3: the GPU suite (range guard, eager fallback, held-out set 2), then the hybrid's
# phase costs (tools/ablate.py variants: base, tail0 = no corrected layer, h8plain = corrected layers
# without the correction terms, noheadv = no in-place right head)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rs > gpurun_out/r04/pytest_gpu_b.log 2>&1
rc=$?; tail -25 gpurun_out/r04/pytest_gpu_b.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ABLATE_ONLY=base,tail0,h8plain,noheadv timeout -k 10 300 python -u tools/ablate.py run f16mix f16-plain > gpurun_out/r04/ablate_hyb.log 2>&1
rc2=$?; cat gpurun_out/r04/ablate_hyb.log | grep -v amdgpu.ids; exit $rc2
