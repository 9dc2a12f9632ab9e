# round 6: A/B of the metric epilogue over long config-4 runs (same box, alternating): RRCDNet and DSDN,
# 2 M spectra each, fused (rdn_forward_metrics) vs forward + metrics kernel, and the graphics clock
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/r06_c4ab}
mkdir -p $OUT
for rep in 1 2; do
  for a in RRCDNet DSDN; do
    for mode in fused unfused; do
      flag=""; [ $mode = unfused ] && flag="--no-fused-metrics"
      timeout -k 10 300 python -u tools/config4.py --total 2000000 --archs $a $flag --out $OUT/c4_${a}_${mode}_$rep.json > $OUT/c4_${a}_${mode}_$rep.log 2>&1
      rc=$?; echo "$rep $a $mode rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/c4_${a}_${mode}_$rep.json'));v=d['networks']['$a'];print(round(v['spectra_per_s']), round(v['seconds'],2))")"
      if [ $rc -ne 0 ]; then tail -3 $OUT/c4_${a}_${mode}_$rep.log; exit $rc; fi
    done
  done
done
