# persistent round recurrence: its GPU tests, then bench lines (c3, c2) with per-phase times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_round_p.py tests/test_gpu_checkpoint.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rp_tests.log 2>&1 && \
bash tools/gpurun/bench_cfgs.sh rp "${1:-c3 c2}" --no-chunked --no-check
