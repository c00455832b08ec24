# ingest kernel variants: parity tests on each, then ms per launch
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sha_var.log
for v in libhgx.so libhgx_exp22.so libhgx_exp23.so; do
  HGX_LIB=$v timeout -k 10 120 python -u -m pytest tests/test_gpu_sha256.py -m gpu -x -q --timeout 100 --timeout-method thread >> gpurun_out/sha_var.log 2>&1 || exit 1
  HGX_LIB=$v timeout -k 10 90 python -u -c "
import bench, json, os
r = bench.ingest_leg(10_000_000, 5, 2, 0)
print(os.environ['HGX_LIB'], r['ms_per_launch'], r['roofline']['frac'])" >> gpurun_out/sha_var.log 2>&1 || exit 1
done
