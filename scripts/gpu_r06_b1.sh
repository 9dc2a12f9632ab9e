# round 6: batch-1 status path through a pinned bounce buffer (abi read_words), the team occupancy
# cache and the module's one status call for every 16-bit network: GPU suite, then the latency split
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_b1}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then tail -30 $OUT/pytest_gpu.log; exit $rc; fi
for a in ADSDN APIDN RRCDNet DSDN; do
  B1_ARCH=$a timeout -k 10 300 python -u tools/batch1_profile.py > $OUT/batch1_$a.log 2>&1
  rc=$?; echo "$a: $(grep -m1 module $OUT/batch1_$a.log)"; if [ $rc -ne 0 ]; then tail -5 $OUT/batch1_$a.log; exit $rc; fi
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['frac'],d.get('batch1'))"; exit $rc
