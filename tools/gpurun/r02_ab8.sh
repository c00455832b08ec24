# A/B of k_cts_tile at 8 waves per SIMD (HGX_CTS_W8): order-path parity under the variant, then both benches
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VAR=${VAR:-exp_w8}
HGX_LIB=libhgx_$VAR.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab8_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab8_base.log 2>&1 && \
HGX_LIB=libhgx_$VAR.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab8_var.log 2>&1
