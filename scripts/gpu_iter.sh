# One GPU iteration: bf16 parity subset, ablation/A-B timing, headline bench.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_forward_gpu.py -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-bf16 and not bf16x3}" > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_iter.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ablate.py run ${ABLATE_DTYPES:-bf16 bf16x3} > gpurun_out/ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 8 > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-1800
