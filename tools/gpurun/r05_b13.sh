# k_cts_tile: the tile's firstDescendants by 16-byte loads through LDS (n <= 256, compact): A/B, tests
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
line() {
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'rounds %.2f order %.2f coords %.2f' % (p['rounds_ms'], p['order_ms'], p['coords_ms']), {x: round(k[x]['ms'],3) for x in ('cts_median','order_sort','round_search','fd_build','la_sweep')})" $1 $2
}
for c in c3 c2; do
  for v in libhgx_b11.so libhgx.so libhgx_b11.so libhgx.so; do
    HGX_LIB=$v timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b13_${c}_$v.json 2> $O/b13_${c}_$v.log || exit $?
    line $O/b13_${c}_$v.json ${c}_$v
  done
done
timeout -k 10 1100 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > $O/b13_tests.log 2>&1 || { tail -40 $O/b13_tests.log; exit 1; }
tail -1 $O/b13_tests.log
