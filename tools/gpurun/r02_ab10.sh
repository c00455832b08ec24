# A/B of the famous-masked WLAT (no fw load in the timestamp gathers): parity of the new default build, then the new (base) and the previous build (var) benches
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VAR=${VAR:-exp_old}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_incremental.py tests/test_gpu_reset.py tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab10_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab10_base.log 2>&1 && \
HGX_LIB=libhgx_$VAR.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab10_var.log 2>&1
