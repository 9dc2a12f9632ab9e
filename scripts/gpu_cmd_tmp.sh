set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forward_gpu.py -x -v --timeout 120 --timeout-method thread -k "f16f8" > gpurun_out/pytest_f16f8.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "trained.*f16f8 max-abs|passed|failed|Error" gpurun_out/pytest_f16f8.log | head -12
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ablate.py run f16f8 > gpurun_out/ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate.log | tail -12
