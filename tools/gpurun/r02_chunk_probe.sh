set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe/chunked_probe.py 256 1000000 1000 0 0 > gpurun_out/chunk1.log 2>&1 && \
timeout -k 10 300 python -u tools/probe/chunked_probe.py 256 1000000 1000 0 1 >> gpurun_out/chunk1.log 2>&1
