# round-path and insert parity tests, then the c3 and c2 benches (no extra legs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_ingest_store.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/q_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ingest --no-chunked > gpurun_out/q_bench_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/q_bench_c2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/q_bench_c4.log 2>&1
