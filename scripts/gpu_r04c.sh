# round 4, call 4: GPU suite (input gate, f64-judged range tests, held-out fp32 criterion) + hybrid phase stamps
# + the faster vectorized head (cur) against the previous tree (base)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rs > gpurun_out/r04/pytest_gpu_c.log 2>&1
rc=$?; tail -12 gpurun_out/r04/pytest_gpu_c.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/hyb_stamps.py > gpurun_out/r04/hyb_stamps.log 2>&1
rc2=$?; grep -v amdgpu.ids gpurun_out/r04/hyb_stamps.log; if [ $rc2 -ne 0 ]; then exit $rc2; fi
ABLATE_ONLY=base,cur timeout -k 10 200 python -u tools/ablate.py run f16mix > gpurun_out/r04/ablate_head.log 2>&1
rc3=$?; grep -v amdgpu.ids gpurun_out/r04/ablate_head.log; exit $rc3
