# A/B of a round-step variant on c2: parity of n = 33..64 cases under the variant, then both benches
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VAR=${VAR:-exp_h1}
HGX_LIB=libhgx_$VAR.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py -x -q --timeout 200 --timeout-method thread -k "64 or 128" > gpurun_out/ab4_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab4_base.log 2>&1 && \
HGX_LIB=libhgx_$VAR.so timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab4_var.log 2>&1
