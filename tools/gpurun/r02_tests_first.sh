# GPU tests first (optionally only the given test files), then one c3 bench line
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ $# -gt 0 ]; then SEL=("$@"); else SEL=(tests); fi
timeout -k 10 780 python -u -m pytest "${SEL[@]}" -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/tests.log 2>&1 && \
timeout -k 10 360 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.log
