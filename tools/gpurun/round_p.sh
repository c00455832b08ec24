# persistent round recurrence: its GPU tests, phase clocks (prof build), then bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_round_p.py tests/test_gpu_checkpoint.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rp_tests.log 2>&1 && \
for c in ${1:-c3 c2}; do HGX_LIB=libhgx_prof.so timeout -k 10 300 python -u tools/phase_timing.py $c 2 > gpurun_out/rp_phases_$c.log 2>&1 || exit $?; done && \
bash tools/gpurun/bench_cfgs.sh rp "${1:-c3 c2}" --no-chunked --no-check
