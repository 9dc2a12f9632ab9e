# Variant parity + timing on one GPU box (tools/ablate.py variants built in the container).
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${PARITY_ARCHS}" != none ]; then
timeout -k 10 300 python -u tools/ablate.py parity ${PARITY_DTYPE:-fp32} ${PARITY_ARCHS} > gpurun_out/ablate_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate_parity.log | tail -40
if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 300 python -u tools/ablate.py run ${ABLATE_DTYPES:-fp32} > gpurun_out/ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate.log | tail -20
exit $rc
