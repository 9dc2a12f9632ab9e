# round 4, call 23: persistent two-pass hybrid (persist: one workgroup per CU over a contiguous run of
# tiles, interior tiles first with the successor's stem inputs issued behind the left head) vs cur
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04
mkdir -p $OUT
ABLATE_ONLY=cur,persist timeout -k 10 200 python -u tools/ablate.py run f16mix > $OUT/ablate_s.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_s.log; if [ $rc -ne 0 ]; then exit $rc; fi
RDN_ABLATE_L=1200 ABLATE_ONLY=cur,persist timeout -k 10 200 python -u tools/ablate.py run f16mix > $OUT/ablate_s1200.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ablate_s1200.log; exit $rc
