# round 6: lastAncestors' time-segment pass in 64-byte column blocks for n in (128, 256] (c3: 8 blocks x 32
# segments instead of 16 x 16): first one c3 line of each build (the kernel's time and whether the exactness
# check held), then the tests through lastAncestors (whole c3 pin included), then the A/B again
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
for L in libhgx_pre.so libhgx.so; do
  HGX_LIB=$L timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline --no-ingest \
    --no-check --no-chunked > $O/la16_c3_${L}_1.json 2> $O/la16_c3_${L}_1.log || { tail -20 $O/la16_c3_${L}_1.log; exit 1; }
  echo "$L $(python tools/r06_summary.py $O/la16_c3_${L}_1.json | cut -c1-700)"
  grep -o "'la_wave_segs': [0-9.]*\|'la_verify': [0-9.]*\|'la_wave_fallbacks': [0-9.]*" $O/la16_c3_${L}_1.log | sort | uniq -c
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_la_wave.py tests/test_gpu_parity.py tests/test_gpu_scale.py \
  tests/test_gpu_full_digests.py tests/test_gpu_incremental.py -x -q --timeout 300 --timeout-method thread \
  > $O/la16_tests.log 2>&1 || { tail -40 $O/la16_tests.log; exit 1; }
tail -1 $O/la16_tests.log
for L in libhgx_pre.so libhgx.so; do
  HGX_LIB=$L timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline --no-ingest \
    --no-check --no-chunked > $O/la16_c3_${L}_2.json 2> $O/la16_c3_${L}_2.log || { tail -20 $O/la16_c3_${L}_2.log; exit 1; }
  echo "$L $(python tools/r06_summary.py $O/la16_c3_${L}_2.json | cut -c1-700)"
done
