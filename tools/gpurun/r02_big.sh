# big-n round step (candidate chunks): round-path parity tests, then the c5 and c3 benches
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_reset.py -x -q --timeout 240 --timeout-method thread > gpurun_out/big_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-ingest --no-chunked > gpurun_out/big_bench_c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/big_bench_c3.log 2>&1
