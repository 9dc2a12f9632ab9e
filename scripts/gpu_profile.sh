# Profiling pass: parity table, rocprofv3 kernel-trace stats per dtype, PMC counter passes.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u tools/parity_report.py --out gpurun_out/parity.md > gpurun_out/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/parity.log; exit $rc; fi
timeout -k 10 60 rocprofv3 -L > gpurun_out/prof/counters.txt 2>&1; echo "list rc=$?"
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for dt in bf16 bf16x3 fp32; do
  B=4096; [ $dt = fp32 ] && B=1024
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$dt -o kt -- python3 $BENCH --dtype $dt --batch $B > gpurun_out/prof/kt_$dt.log 2>&1
  rc=$?; echo "kt $dt rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof/kt_$dt.log; exit $rc; fi
done
for dt in bf16 bf16x3; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/pmc1_$dt -o p -- python3 $BENCH --dtype $dt --batch 2048 > gpurun_out/prof/pmc1_$dt.log 2>&1
  rc=$?; echo "pmc1 $dt rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof/pmc1_$dt.log; exit $rc; fi
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/prof/pmc_$ctr -o p -- python3 $BENCH --dtype bf16x3 --batch 2048 > gpurun_out/prof/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof/pmc_$ctr.log; exit $rc; fi
done
