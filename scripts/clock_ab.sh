# Effective clock + MFMA busy of ablation variants (tools/ablate.py, one process per variant):
#   ABLATE_VARIANTS="base m32" ABLATE_DTYPE=f16 bash scripts/clock_ab.sh
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/clock
for v in ${ABLATE_VARIANTS:-base m32}; do
  ABLATE_ONLY=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d gpurun_out/clock/$v -o p -- python3 tools/ablate.py run ${ABLATE_DTYPE:-f16} > gpurun_out/clock/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; grep -v amdgpu.ids gpurun_out/clock/$v.log | tail -2
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/clock_summary.py gpurun_out/clock/*/
