# round 4, call 20: the stem's taps -1 / +1 from DPP wave shifts of the lanes' own x (NK + 2 loads per
# lane instead of 3 NK; sdpp = this tree, prev = the last commit), stamps, the GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
ABLATE_ONLY=prev,sdpp timeout -k 10 200 python -u tools/ablate.py run f16mix f16-plain > $OUT/ablate_q.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_q.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/hyb_stamps.py > $OUT/hyb_stamps_q.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/hyb_stamps_q.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_q.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $OUT/pytest_gpu_q.log | tail -12; exit $rc
