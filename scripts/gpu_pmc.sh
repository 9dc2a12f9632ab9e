# PMC passes over one short bench run of a single dtype (each pass its own process; gfx950 slot limits).
#   bash scripts/gpu_pmc.sh <dtype> <batch> <outdir>
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
DT=${1:-bf16}; B=${2:-2048}; OUT=${3:-gpurun_out/pmc_$DT}
mkdir -p $OUT
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --dtype $DT --batch $B"
[ -f $OUT/counters.txt ] || timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o p -- python3 $BENCH > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc ($CTRS)"; if [ $rc -ne 0 ]; then tail -3 $OUT/p$i.log; exit $rc; fi
done <<'LIST'
SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU
SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT
LIST
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $BENCH > $OUT/kt.log 2>&1
echo "kt rc=$?"
