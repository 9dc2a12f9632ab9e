# round 5: PIDN walk -- parity (golden + bitwise vs tiles), A/B at L = 10,000 and 16,384
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05j
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_forward_gpu.py -x -q --timeout 120 --timeout-method thread -k "walk or short_tiles" > $OUT/pytest_walk.log 2>&1
rc=$?; tail -2 $OUT/pytest_walk.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_walk.log | head -30; exit $rc; fi
timeout -k 10 300 python -u tools/walk_ab.py PIDN:f16 DSDN:f16 > $OUT/walk_ab.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/walk_ab.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/walk_ab.py --batch 2500 --L 16384 PIDN:f16 > $OUT/walk_ab_16k.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/walk_ab_16k.log; exit $rc
