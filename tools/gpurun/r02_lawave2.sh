# dataflow lastAncestors pass: parity, then timing
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_la_wave.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/lawave_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
