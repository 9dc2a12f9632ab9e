# Weight-stream diagnostics of the ping-pong engine: ablation variants + L1/TA counters (f16-plain RRCDNet).
set +e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ablate.py run f16 > gpurun_out/ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate.log | tail -6
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr TA_TA_BUSY_sum --output-format csv -d gpurun_out/tcp -o p -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-pipeline --no-batch1 --dtype f16-plain --batch 2048 > gpurun_out/tcp.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -2 gpurun_out/tcp.log | cut -c1-300
