# Round evidence that does not depend on kernel tuning: parity table (incl. the held-out set),
# config-1 records (test.npz, N = 1000, engine vs the reference CPU path), config-4 at one rank's
# share of 100 M spectra, all-network throughput.  STAGES selects (default: parity config1 throughput).
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03
mkdir -p $OUT
STAGES=${STAGES:-parity config1 throughput}
for st in $STAGES; do
  case $st in
    parity)
      timeout -k 10 400 python -u tools/parity_report.py --out $OUT/parity_table.md > $OUT/parity.log 2>&1
      rc=$?; echo "parity rc=$rc"; grep -E "held-out|RRCDNet \| trained \| f16 " $OUT/parity.log
      if [ $rc -ne 0 ]; then tail -5 $OUT/parity.log; exit $rc; fi ;;
    config1)
      for spec in "DenoiseCNN fp32" "RRCDNet f16" "RRCDNet fp32"; do
        set -- $spec
        timeout -k 10 600 python -u tools/config1_eval.py --n 1000 --cpu-n ${CPU_N:-1000} --arch $1 --dtype $2 \
          --out $OUT/config1_$1_$2.json > $OUT/config1_$1_$2.log 2>&1
        rc=$?; echo "config1 $1 $2 rc=$rc"; grep -E "max_|spectra_per_s" $OUT/config1_$1_$2.json
        if [ $rc -ne 0 ]; then tail -5 $OUT/config1_$1_$2.log; exit $rc; fi
      done ;;
    config4)
      timeout -k 10 1000 python -u tools/config4.py --total ${C4_TOTAL:-12500000} --out $OUT/config4_shard.json \
        > $OUT/config4.log 2>&1
      rc=$?; echo "config4 rc=$rc"; tail -1 $OUT/config4.log | cut -c1-1500
      if [ $rc -ne 0 ]; then exit $rc; fi ;;
    throughput)
      timeout -k 10 600 python -u tools/throughput_table.py --out $OUT/throughput.md > $OUT/throughput.log 2>&1
      rc=$?; echo "throughput rc=$rc"; grep -E "ADSDN|APIDN|RRCDNet \| 10000 \| f16 " $OUT/throughput.md | grep -E "\| f16 \|"
      if [ $rc -ne 0 ]; then tail -3 $OUT/throughput.log; exit $rc; fi ;;
  esac
done
