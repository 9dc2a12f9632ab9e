# round 5: the RDN_F16MIX walk at 576 rows (4.5 in-place blocks) -- parity, A/B against 512
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05f
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_forward_gpu.py -x -v --timeout 120 --timeout-method thread -k "walk" > $OUT/pytest_walk.log 2>&1
rc=$?; tail -2 $OUT/pytest_walk.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_walk.log | head -30; exit $rc; fi
RDN_WALK=1 ABLATE_ONLY=base,mix512 RDN_ABLATE_ARCH=RRCDNet timeout -k 10 300 python -u tools/ablate.py run f16 > $OUT/ablate_mix.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_mix.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/walk_ab.py RRCDNet:f16 > $OUT/walk_ab.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/walk_ab.log; exit $rc
