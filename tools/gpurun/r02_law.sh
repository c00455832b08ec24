# lastAncestors wavefront above 896 chains: la_wave tests, big-n parity, c5 bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_la_wave.py -x -q --timeout 240 --timeout-method thread > gpurun_out/law_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py -x -q --timeout 240 --timeout-method thread -k "1000 or 1024" > gpurun_out/law_tests2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-ingest --no-chunked > gpurun_out/law_bench_c5.log 2>&1
