# round 4, call 2: resume the held-out RRCDNet training to the reference's 200 epochs (28,200 steps of
# batch 32 over 4,500 spectra), then the GPU suite on the range-guard build
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/heldout2 gpurun_out/r04
cp scratch/heldout2/ckpt.pt gpurun_out/heldout2/ 2>/dev/null
timeout -k 10 560 python -u tests/golden/train_heldout_gpu.py --out gpurun_out/heldout2 --steps 28200 --max-seconds 520 \
  > gpurun_out/heldout2/train2.log 2>&1
rc=$?; tail -3 gpurun_out/heldout2/train2.log; echo "train rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 124 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu_a.log 2>&1
rc=$?; tail -15 gpurun_out/r04/pytest_gpu_a.log; exit $rc
