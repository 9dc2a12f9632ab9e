# Final evidence on the committed tree, in ONE session: the default bench line,
# the rocprofv3 kernel trace of the same bench (the dominant kernel's average must not exceed that
# line's ms_per_step), PMC passes (separate processes, gfx950 slot limits) for the headline hybrid,
# plain f16, and the CBAM team kernels (ADSDN / APIDN 'f16').
#   then, on the build host: python tools/summarize_profiles.py <OUT> profiles/r06
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/final}
mkdir -p $OUT
STAGES=${STAGES:-bench kt pmc}
if [[ " $STAGES " == *" bench "* ]]; then
  timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi
  grep "^{" $OUT/bench.log | tail -1 > $OUT/bench.json
fi
if [[ " $STAGES " == *" kt "* ]]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --no-cpu-baseline --no-configs --sustained-seconds 0 > $OUT/kt_bench.log 2>&1
  rc=$?; echo "kt rc=$rc"; tail -1 $OUT/kt_bench.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi
  grep "^{" $OUT/kt_bench.log | tail -1 > $OUT/kt_bench.json
fi
# PMC: the timed launches only (no batch-1 loop, variants, pipeline or configs)
SHORT="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-pipeline --no-batch1 --no-configs --sustained-seconds 0"
if [[ " $STAGES " == *" pmc "* ]]; then
  for spec in ${PROFILE_SPECS:-RRCDNet:f16:8192 RRCDNet:f16-plain:8192 ADSDN:f16:2048 APIDN:f16:2048}; do
    IFS=: read -r arch dt bsz <<< "$spec"
    for ctr in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" "SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"; do
      tag=$(echo $ctr | cut -d' ' -f1)
      timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/pmc_${arch}-${dt}_$tag -o p -- python3 $SHORT --arch $arch --dtype $dt --batch $bsz > $OUT/pmc_${arch}-${dt}_$tag.log 2>&1
      rc=$?; echo "pmc $arch $dt $tag rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/pmc_${arch}-${dt}_$tag.log; exit $rc; fi
    done
  done
fi
