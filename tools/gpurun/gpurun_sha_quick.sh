# SHA-256 parity tests + device-resident throughput of the ingest kernel only
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sha256.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/shaq_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "
import bench, json
print(json.dumps(bench.ingest_leg(10_000_000, 5, 2, 0)))" > gpurun_out/shaq.json 2> gpurun_out/shaq.log
