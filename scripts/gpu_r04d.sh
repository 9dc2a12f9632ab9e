# round 4, call 5: hybrid head/stem prefetch A/B (base = round-3 tree + range guard, cur2 = this tree,
# prev = in-place-engine-only diagnostic), phase stamps of this tree, then the headline + range tests
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04
ABLATE_ONLY=base,cur2,prev timeout -k 10 200 python -u tools/ablate.py run f16mix > gpurun_out/r04/ablate_d.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04/ablate_d.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/hyb_stamps.py > gpurun_out/r04/hyb_stamps_d.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04/hyb_stamps_d.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests/test_range_gpu.py tests/test_headline_gpu.py tests/test_forward_gpu.py -m gpu -q -s --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu_d.log 2>&1
rc=$?; grep -E "heldout|config 1|passed|failed" gpurun_out/r04/pytest_gpu_d.log | tail -30; exit $rc
