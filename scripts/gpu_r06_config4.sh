# round 6: config 4 at its stated scale per rank with the metric epilogue (rdn_forward_metrics): 100 M
# spectra over 8 GPUs is 12.5 M per rank; rank 0 owns indices [0, 12.5 M), which this one-GPU run
# processes (W = 1, --total 12,500,000), each network its own process
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/r06_config4}
mkdir -p $OUT
for a in RRCDNet DSDN ADSDN; do
  timeout -k 10 400 python -u tools/config4.py --total 12500000 --archs $a --out $OUT/config4_12p5M_$a.json > $OUT/config4_$a.log 2>&1
  rc=$?; echo "$a rc=$rc"; tail -1 $OUT/config4_$a.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi
done
