# full GPU suite, then the default bench line
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u tools/probe/chunk_calls.py 256 1000000 1000 > gpurun_out/chunk_calls.log 2>&1
