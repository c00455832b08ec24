# GPU parity tests (optionally filtered by $1), then one c3 bench line with per-kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K=${1:-}
if [ -n "$K" ]; then SEL=(-k "$K"); else SEL=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${SEL[@]}" > gpurun_out/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.log
