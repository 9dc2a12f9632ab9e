# Quick GPU measurement pass: headline bench (all dtypes) + in-place kernel ablation, one process each.
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 8 > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-1500
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -d tools/ablate_build ]; then
  timeout -k 10 300 python -u tools/ablate.py run ${ABLATE_DTYPES:-bf16x3 bf16} > gpurun_out/ablate.log 2>&1
  rc=$?; echo "ablate rc=$rc"; cat gpurun_out/ablate.log | grep -v amdgpu.ids
fi
