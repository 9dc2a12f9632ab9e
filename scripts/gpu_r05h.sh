# round 5: batch-1 call breakdown
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 300 python -u tools/batch1_profile.py > $OUT/batch1.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/batch1.log | head -45; exit $rc
