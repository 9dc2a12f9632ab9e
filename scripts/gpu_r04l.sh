# round 4, call 13: the tail range vote on the combine barrier (comb = this tree, vote = call 12), GPU suite, smoke
# no LDS vote words, one barrier fewer; vote = this tree, stg = call 11's), stamps, the GPU suite, smoke
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
ABLATE_ONLY=vote,comb timeout -k 10 200 python -u tools/ablate.py run f16mix > $OUT/ablate_l.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_l.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/hyb_stamps.py > $OUT/hyb_stamps_l.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/hyb_stamps_l.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > $OUT/pytest_gpu_l.log 2>&1
rc=$?; grep -E "heldout|config 1|passed|failed|Error" $OUT/pytest_gpu_l.log | tail -12; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_l.log 2>&1
rc=$?; tail -2 $OUT/smoke_l.log; exit $rc
