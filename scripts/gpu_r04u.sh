# round 4, call 25: instruction-cache counters of the hybrid (419 KB of code) vs plain f16; one copy of
# the ping-pong layer per loop (oneloop) vs cur; the module-path GPU tests after the range-word read change
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
timeout -k 10 400 bash scripts/pmc_icache.sh
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
ABLATE_ONLY=cur,oneloop timeout -k 10 200 python -u tools/ablate.py run f16mix > $OUT/ablate_u.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_u.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_range_gpu.py tests/test_evaluate_gpu.py tests/test_headline_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_u.log 2>&1
rc=$?; tail -1 $OUT/pytest_u.log; exit $rc
