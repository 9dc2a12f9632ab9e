# round 4, call 7: the e2m3 MFMA's rate in the corrected tail (f6: the correction MFMA with fp6
# format flags, wrong results -- an upper bound for an fp6 correction), against the product tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04
ABLATE_ONLY=cur,f6,h8plain,tail0 timeout -k 10 200 python -u tools/ablate.py run f16mix f16f8 > gpurun_out/r04/ablate_f.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04/ablate_f.log; exit $rc
