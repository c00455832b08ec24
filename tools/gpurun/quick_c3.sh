# quick check after a kernel change: parity subset, then c3 phase times and one bench line
# usage: bash tools/gpurun/quick_c3.sh TAG "pytest -k expression"
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-q}; K=${2:-gossip_batch or kat or fixture or incremental or int32}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log && grep "kernel profile" gpurun_out/${TAG}_bench.log
