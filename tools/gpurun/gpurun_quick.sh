# quick GPU iteration: parity tests (optionally filtered by $1) then a c3 bench with per-kernel times
set -o pipefail
mkdir -p gpurun_out
K=${1:-gossip or fixture or batched or core}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/q_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.log
