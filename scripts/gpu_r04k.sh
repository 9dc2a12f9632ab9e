# round 4, call 12: the spiked-tile vote from each wave's own ballot (every wave reads all the tile's x:
# no LDS vote words, one barrier fewer; vote = this tree, stg = call 11's), stamps, the GPU suite, smoke
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
ABLATE_ONLY=stg,vote timeout -k 10 200 python -u tools/ablate.py run f16mix > $OUT/ablate_k.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_k.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/hyb_stamps.py > $OUT/hyb_stamps_k.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/hyb_stamps_k.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > $OUT/pytest_gpu_k.log 2>&1
rc=$?; grep -E "heldout|config 1|passed|failed|Error" $OUT/pytest_gpu_k.log | tail -12; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_k.log 2>&1
rc=$?; tail -2 $OUT/smoke_k.log; exit $rc
