# incremental-schedule tests + parity, then the chunked per-call probe
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_parity.py tests/test_gpu_ingest_store.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/probe/chunked_probe.py 64 200000 1000 > gpurun_out/chunk1.log 2>&1 && \
timeout -k 10 300 python -u tools/probe/chunked_probe.py 256 1000000 1000 >> gpurun_out/chunk1.log 2>&1
