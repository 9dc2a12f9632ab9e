# round 4, call 9: the right head on the MFMA (mhead = this tree, cur = the VGPR-rows head), phase
# stamps, the in-place diagnostics on f16f8 (nostore / nobar / nocread / nosplit / f6: one component
# dropped each, wrong results), the GPU suite, then PMC on f16f8 and the hybrid
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r04
mkdir -p $OUT
ABLATE_ONLY=cur,mhead timeout -k 10 200 python -u tools/ablate.py run f16mix > $OUT/ablate_h.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_h.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/hyb_stamps.py > $OUT/hyb_stamps_h.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/hyb_stamps_h.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > $OUT/pytest_gpu_h.log 2>&1
rc=$?; grep -E "heldout|config 1|passed|failed|Error" $OUT/pytest_gpu_h.log | tail -30; if [ $rc -ne 0 ]; then exit $rc; fi
ABLATE_ONLY=cur,nostore,nobar,nocread,nosplit,f6 timeout -k 10 300 python -u tools/ablate.py run f16f8 > $OUT/ablate_h_diag.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_h_diag.log; if [ $rc -ne 0 ]; then exit $rc; fi
SHORT="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-pipeline --no-batch1 --no-configs"
for dt in f16f8 f16; do
  for ctr in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"; do
    tag=$(echo $ctr | cut -d' ' -f1)
    timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/pmc_h_${dt}_$tag -o p -- python3 $SHORT --arch RRCDNet --dtype $dt --batch 2048 > $OUT/pmc_h_${dt}_$tag.log 2>&1
    rc=$?; echo "pmc $dt $tag rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/pmc_h_${dt}_$tag.log; exit $rc; fi
  done
done
