# dataflow lastAncestors pass: parity first, then timing
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_la_wave.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/lawave_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_reset.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/parity.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u tools/probe/chunk_calls.py 256 1000000 1000 > gpurun_out/chunk_calls.log 2>&1
