# round 6: the order's parts only from 16 MB of order (c2's 4 MB order back on the direct writes): the tests
# through the bucket sort, then c2 / c3 / c4 lines of the new build beside the parts-everywhere build (libhgx_pre.so
# is the build before the parts)
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_seg.py tests/test_gpu_full_config.py tests/test_gpu_insert_and_run.py \
  tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $O/sp2_tests.log 2>&1 \
  || { tail -40 $O/sp2_tests.log; exit 1; }
tail -1 $O/sp2_tests.log
for c in c2 c3 c4; do
  for L in libhgx_pre.so libhgx.so; do
    HGX_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-ingest \
      --no-check --no-chunked > $O/sp2_${c}_${L}.json 2> $O/sp2_${c}_${L}.log || { tail -20 $O/sp2_${c}_${L}.log; exit 1; }
    echo "$L $(python tools/r06_summary.py $O/sp2_${c}_${L}.json | cut -c1-700)"
  done
done
