# A/B of 32-row firstDescendants tiles above 512 chains (HGX_FD_FT32): big-n parity under the variant, then c5 benches
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VAR=${VAR:-exp_ft32}
HGX_LIB=libhgx_$VAR.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_la_wave.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab11_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab11_base.log 2>&1 && \
HGX_LIB=libhgx_$VAR.so timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab11_var.log 2>&1
