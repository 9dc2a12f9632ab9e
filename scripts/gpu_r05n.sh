# round 5: CBAM team16 phase stamps (ADSDN L=10000, APIDN L=10000 and 16384)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05n
mkdir -p $OUT
for spec in ${SPECS:-ADSDN:10000 APIDN:16384}; do
  IFS=: read -r a L <<< "$spec"
  timeout -k 10 200 python -u tools/team_stamps.py $a f16 $L stamps > $OUT/stamps_${a}_$L.log 2>&1
  rc=$?; grep -v amdgpu.ids $OUT/stamps_${a}_$L.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
