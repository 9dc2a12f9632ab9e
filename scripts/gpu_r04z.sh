# round 4, call 30: forward throughput of every network x engine dtype (tools/throughput_table.py) on
# the final tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u tools/throughput_table.py --out gpurun_out/r04/throughput.md > gpurun_out/r04/throughput.log 2>&1
rc=$?; tail -40 gpurun_out/r04/throughput.md; exit $rc
