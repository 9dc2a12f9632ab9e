# round 6 evidence on the final tree, in two calls (each under gpurun's 20-minute limit):
#   PART=a: GPU suite, smoke, parity table, the default bench line and its rocprofv3 kernel trace
#   PART=b: PMC passes (scripts/gpu_final.sh pmc), the all-network throughput table, and the
#           SQ_VALU_MFMA_COEXEC_CYCLES A/B of the static-priority knob (tools/ablate_build base vs prio)
# then, on the build host: python tools/summarize_profiles.py gpurun_out/final6 profiles/r06
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/final6}
mkdir -p $OUT
if [ "${PART:-a}" = a ]; then
  STAGES="tests smoke parity bench kt" OUT=$OUT bash scripts/gpu.sh
  exit $?
fi
STAGES="pmc throughput" OUT=$OUT bash scripts/gpu.sh || exit $?
for ctr in "SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  RDN_ALLOW_STALE_LIB=1 RDN_WALK=1 ABLATE_ONLY=base,prio RDN_ABLATE_ARCH=RRCDNet timeout -s KILL 180 \
    rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/coexec_$tag -o p -- python3 tools/ablate.py run f16-plain \
    > $OUT/coexec_$tag.log 2>&1
  rc=$?; echo "coexec $tag rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/coexec_$tag.log; exit $rc; fi
done
