# LDS bank-conflict attribution for the in-place f16f8 kernel (diagnostic): one PMC pass per
# ablation variant (tools/ablate.py build base nostore h8plain first)
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lds
mkdir -p $OUT
for v in base nostore h8plain; do
  ABLATE_ONLY=$v timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CU_CYCLES --output-format csv -d $OUT/$v -o p -- python3 tools/ablate.py run f16f8 f16mix > $OUT/$v.log 2>&1
  echo "$v ok"
done
