set -e
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pmc3
mkdir -p $OUT
SHORT="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-pipeline --dtype f16-plain"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $SHORT > $OUT/kt.log 2>&1
echo kt ok
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/p1 -o p -- python3 $SHORT > $OUT/p1.log 2>&1
echo p1 ok
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/p2 -o p -- python3 $SHORT > $OUT/p2.log 2>&1
echo p2 ok
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_IFETCH SQ_WAVES --output-format csv -d $OUT/p3 -o p -- python3 $SHORT > $OUT/p3.log 2>&1
echo p3 ok
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $OUT/p4 -o p -- python3 $SHORT > $OUT/p4.log 2>&1 || echo p4 failed
