# ingest kernel variants (waves per SIMD / register prefetch): parity sample + ms per launch
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sha_var.log
for v in libhgx.so libhgx_exp40.so libhgx_exp50.so libhgx_exp60.so; do
  HGX_LIB=$v timeout -k 10 90 python -u -c "
import bench, json, os
r = bench.ingest_leg(10_000_000, 5, 2, 0)
print(os.environ['HGX_LIB'], r['ms_per_launch'], r['roofline']['frac'])" >> gpurun_out/sha_var.log 2>&1 || exit 1
done
