# round 6: the order's finish fused into the bucket sort (k_seg_sort + SortFinish): the tests through the
# bucket sort (full c2 / c4 / c3 / c5 pins included), then c3 / c2 / c4 lines against the previous build, twice
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_sort_seg.py tests/test_gpu_full_config.py tests/test_gpu_full_digests.py \
  tests/test_gpu_scale.py tests/test_gpu_incremental.py -x -q --timeout 300 --timeout-method thread > $O/fin_tests.log 2>&1 \
  || { tail -40 $O/fin_tests.log; exit 1; }
tail -1 $O/fin_tests.log
for rep in 1 2; do
  for c in c3 c2 c4; do
    for L in libhgx_old.so libhgx.so; do
      HGX_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-ingest \
        --no-check --no-chunked > $O/fin_${c}_${L}_$rep.json 2> $O/fin_${c}_${L}_$rep.log || { tail -20 $O/fin_${c}_${L}_$rep.log; exit 1; }
      python -c "import json; d=json.loads([l for l in open('$O/fin_${c}_${L}_$rep.json') if l.startswith('{')][-1]); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print('$rep $L $c', round(d['ms_per_step'],3), 'hbm', round(d['hbm_resident']['ms_per_step'],3), 'order_ms', round(p['order_ms'],3), 'sort', round(k['order_sort']['ms'],3))"
    done
  done
done
