# one c3 bench line first (fast signal), then the GPU parity tests (optionally filtered by $1)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K=${1:-}
if [ -n "$K" ]; then SEL=(-k "$K"); else SEL=(); fi
timeout -k 10 360 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.log && \
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${SEL[@]}" > gpurun_out/tests.log 2>&1
