# the whole GPU suite on the current build
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/suite.log 2>&1 || { tail -40 gpurun_out/r05/suite.log; exit 1; }
tail -3 gpurun_out/r05/suite.log
