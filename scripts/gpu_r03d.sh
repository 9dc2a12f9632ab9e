set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 500 python -u tools/f16mix_spike_eval.py > gpurun_out/r03/f16mix_spike_eval.log 2>&1
rc=$?; echo "spike eval rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/f16mix_spike_eval.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in stamps alledge; do
timeout -k 10 120 python -u tools/team_stamps.py ADSDN f16 10000 $v > gpurun_out/r03/stamps16_$v.log 2>&1
rc=$?; echo "stamps $v rc=$rc"; grep -E "tile  0|tile  1:|tile  7|tile 15|spectra/s" gpurun_out/r03/stamps16_$v.log
if [ $rc -ne 0 ]; then exit $rc; fi
done
