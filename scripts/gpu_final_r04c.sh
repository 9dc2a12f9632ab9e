# round 4 final evidence on the final tree: GPU suite, smoke, parity table (tools/parity_report.py),
# the default bench line and the rocprofv3 kernel trace of the same bench command, then the PMC passes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/final/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/final/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/parity_report.py --out gpurun_out/final/parity.md > gpurun_out/final/parity.log 2>&1
rc=$?; tail -3 gpurun_out/final/parity.md; if [ $rc -ne 0 ]; then exit $rc; fi
STAGES="bench kt pmc" bash scripts/gpu_final.sh
