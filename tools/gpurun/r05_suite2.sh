# full GPU suite on the packed-columns build, then the default bench line
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite2.log 2>&1 || { tail -40 $O/gpu_suite2.log; exit 1; }
tail -1 $O/gpu_suite2.log
