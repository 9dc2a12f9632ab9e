set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/f16mix_select.py ${SELECT_ARGS} > gpurun_out/f16mix_select.log 2>&1
rc=$?; echo "select rc=$rc"; grep -v amdgpu.ids gpurun_out/f16mix_select.log | tail -20
exit $rc
