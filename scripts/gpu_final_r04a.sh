# round 4 final evidence, part 1: the GPU suite and smoke on the committed tree, then the default bench
# line and the rocprofv3 kernel trace of the same bench command (scripts/gpu_final.sh stages bench, kt)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/final/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/final/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
STAGES="bench kt" bash scripts/gpu_final.sh
