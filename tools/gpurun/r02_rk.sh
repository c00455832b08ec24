# round-path parity tests, phase clocks, c3 + c2 bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_reset.py tests/test_gpu_scale.py tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rk_tests.log 2>&1 && \
HGX_LIB=libhgx_prof.so timeout -k 10 200 python -u tools/phase_timing.py c3 2 > gpurun_out/rk_phases.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ingest --no-chunked > gpurun_out/rk_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/rk_bench_c2.log 2>&1
