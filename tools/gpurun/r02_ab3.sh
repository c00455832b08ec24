# A/B of a round-step variant: parity of the round paths under the variant, phase clocks, c3/c2 bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VAR=${VAR:-exp_xw}
HGX_LIB=libhgx_$VAR.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab3_tests.log 2>&1 && \
HGX_LIB=libhgx_prof.so timeout -k 10 200 python -u tools/phase_timing.py c3 1 > gpurun_out/ab3_phases_base.log 2>&1 && \
HGX_LIB=libhgx_${VAR}prof.so timeout -k 10 200 python -u tools/phase_timing.py c3 1 > gpurun_out/ab3_phases_var.log 2>&1 && \
for cfg in c3 c2; do
timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab3_base_$cfg.log 2>&1 && \
HGX_LIB=libhgx_$VAR.so timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab3_var_$cfg.log 2>&1 || exit 1
done
