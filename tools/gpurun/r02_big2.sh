# big-n round step: n > 256 parity cases, c5 bench, c5 phase clocks
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_reset.py -x -q --timeout 240 --timeout-method thread -k "300 or 512 or 600 or 1000 or 1024" > gpurun_out/big_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-ingest --no-chunked > gpurun_out/big_bench_c5.log 2>&1 && \
HGX_LIB=libhgx_prof.so timeout -k 10 200 python -u tools/phase_timing.py c5 2 > gpurun_out/c5_phases.log 2>&1
