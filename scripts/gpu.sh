# One parametrised GPU lease script (replaces the per-lease scripts of rounds 3-5).
#
#   STAGES="ab tests" OUT=gpurun_out/r06a bash scripts/gpu.sh
#
# Stages (run in the order listed here; the script stops at the first failing stage):
#   ab          tools/ablate.py A/B of the prebuilt variants in tools/ablate_build (AB_VARIANTS, comma list;
#               AB_SPECS = arch:dtype pairs; AB_L = spectrum lengths), one process per (spec, L)
#   stamps      phase stamps of the hybrid walk (tools/hyb_stamps.py, a -DRDN_HYB_STAMPS=1 build)
#   tests       the GPU suite (PYTEST_K: a -k expression)
#   smoke       __graft_entry__.smoke()
#   parity      tools/parity_report.py
#   bench kt pmc  scripts/gpu_final.sh (the bench line, its rocprofv3 kernel trace, PMC passes)
#   throughput  tools/throughput_table.py
# Every GPU step runs under its own timeout; after a failure nothing else runs on the GPU.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/lease}
mkdir -p "$OUT"
STAGES=${STAGES:-tests}
has() { [[ " $STAGES " == *" $1 "* ]]; }

if has ab; then
  for L in ${AB_L:-10000}; do
    for spec in ${AB_SPECS:-RRCDNet:f16 RRCDNet:f16-plain DenoiseCNN:f16}; do
      IFS=: read -r arch dt <<< "$spec"
      log=$OUT/ab_${arch}_${dt}_$L.log
      RDN_ALLOW_STALE_LIB=1 RDN_WALK=${AB_WALK:-1} RDN_ABLATE_L=$L ABLATE_ONLY=${AB_VARIANTS:-base} RDN_ABLATE_ARCH=$arch \
        timeout -k 10 300 python -u tools/ablate.py run $dt $dt > $log 2>&1
      rc=$?; echo "ab $arch $dt L=$L rc=$rc"; grep -v amdgpu.ids $log | tail -40; if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
fi
if has stamps; then
  RDN_WALK=1 timeout -k 10 300 python -u tools/hyb_stamps.py > $OUT/hyb_stamps.log 2>&1
  rc=$?; grep -v amdgpu.ids $OUT/hyb_stamps.log | tail -20; if [ $rc -ne 0 ]; then exit $rc; fi
fi
if has tests; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -1 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|^E " $OUT/pytest_gpu.log | head -30; exit $rc; fi
fi
if has smoke; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; tail -1 $OUT/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
fi
if has parity; then
  timeout -k 10 300 python -u tools/parity_report.py --out $OUT/parity.md > $OUT/parity.log 2>&1
  rc=$?; tail -2 $OUT/parity.md; if [ $rc -ne 0 ]; then exit $rc; fi
fi
INNER="$(echo "$STAGES" | tr ' ' '\n' | grep -x 'bench\|kt\|pmc' | tr '\n' ' ')"
if [ -n "$INNER" ]; then
  OUT=$OUT STAGES="$INNER" bash scripts/gpu_final.sh
  rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
fi
if has throughput; then
  timeout -k 10 400 python -u tools/throughput_table.py --out $OUT/throughput.md > $OUT/throughput.log 2>&1
  rc=$?; tail -3 $OUT/throughput.log; exit $rc
fi
