# SHA-256 parity tests then a c3 bench line with the ingest side leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sha256.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/sha_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sha_bench.json 2> gpurun_out/sha_bench.log
