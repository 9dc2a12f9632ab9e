# Instruction-cache counters of the headline hybrid vs plain f16 (diagnostic): one pass each
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r04/icache
mkdir -p $OUT
SHORT="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-variants --no-pipeline --no-batch1 --no-configs --batch 4096"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -o "SQC_[A-Z_]*" $OUT/counters.txt | sort -u > $OUT/sqc.txt
cat $OUT/sqc.txt | tr '\n' ' '; echo
for dt in f16 f16-plain; do
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $OUT/pmc_$dt -o p -- python3 $SHORT --dtype $dt > $OUT/pmc_$dt.log 2>&1
  rc=$?; echo "pmc $dt rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/pmc_$dt.log; exit $rc; fi
done
