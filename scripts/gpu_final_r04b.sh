# round 4 final evidence, part 2: the PMC passes (scripts/gpu_final.sh stage pmc: FETCH_SIZE, WRITE_SIZE
# and two SQ groups, each its own process) for the hybrid, plain f16 and the CBAM team kernels
set -o pipefail
cd "$(dirname "$0")/.."
STAGES="pmc" bash scripts/gpu_final.sh
