# Profiling pass for the round's evidence (profiles/): parity table, the headline bench under
# rocprofv3 --kernel-trace --stats (the same default command the driver runs), and separate PMC
# passes (FETCH_SIZE, WRITE_SIZE, SQ counters) per MI355X_MICROARCH.md §HBM / §PMC slots.
# STAGES selects a subset (default: parity kt pmc throughput).
# Afterwards, on the build host: python tools/summarize_profiles.py gpurun_out/prof profiles/rNN
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
STAGES=${STAGES:-parity kt pmc throughput}
if [[ " $STAGES " == *" parity "* ]]; then
  timeout -k 10 300 python -u tools/parity_report.py --out $OUT/parity.md > $OUT/parity.log 2>&1
  rc=$?; echo "parity rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/parity.log; exit $rc; fi
fi
if [[ " $STAGES " == *" kt "* ]]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py > $OUT/kt_bench.log 2>&1
  rc=$?; echo "kt rc=$rc"; tail -1 $OUT/kt_bench.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi
fi
# PMC passes: the timed launches only (batch 8192; no batch-1 loop, no variants, no pipeline), so
# the per-dispatch averages are those of the headline launch
SHORT="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-pipeline --no-batch1"
if [[ " $STAGES " == *" pmc "* ]]; then
  for dt in ${PROFILE_DTYPES:-f16 f16-plain f16f8}; do
    for ctr in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"; do
      tag=$(echo $ctr | cut -d' ' -f1)
      timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_${dt}_$tag -o p -- python3 $SHORT --dtype $dt > $OUT/pmc_${dt}_$tag.log 2>&1
      rc=$?; echo "pmc $dt $tag rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/pmc_${dt}_$tag.log; exit $rc; fi
    done
  done
fi
if [[ " $STAGES " == *" throughput "* ]]; then
  timeout -k 10 400 python -u tools/throughput_table.py --out $OUT/throughput.md > $OUT/throughput.log 2>&1
  rc=$?; echo "throughput rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/throughput.log; exit $rc; fi
fi
