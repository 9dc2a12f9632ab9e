# round 4, call 6: hybrid A/B (cur2 = call-5 tree, cur = this tree: left-stem loads behind the head's
# weights, right-head rows in VGPRs, L2 touch of the next tile's x; park / touch0 / touch512 revert
# one change each), phase stamps, then the headline + range + forward tests
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04
ABLATE_ONLY=base,cur2,cur,park,touch0,touch512 timeout -k 10 240 python -u tools/ablate.py run f16mix > gpurun_out/r04/ablate_e.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04/ablate_e.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/hyb_stamps.py > gpurun_out/r04/hyb_stamps_e.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04/hyb_stamps_e.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests/test_range_gpu.py tests/test_headline_gpu.py tests/test_forward_gpu.py tests/test_pipeline_gpu.py -m gpu -q -s --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu_e.log 2>&1
rc=$?; grep -E "heldout|config 1|passed|failed" gpurun_out/r04/pytest_gpu_e.log | tail -30; exit $rc
