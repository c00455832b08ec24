# full GPU suite, chunked probe, c3 bench with the chunked leg
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/ch_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/probe/chunk_calls.py 256 1000000 1000 > gpurun_out/chunk_calls.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-ingest > gpurun_out/ch_bench.log 2>&1
