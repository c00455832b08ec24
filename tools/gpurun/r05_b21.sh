# k_cts_pair (a thread per pair of events) against k_cts_tile (HGX_CTS_PAIR=0): c3 c2 A/B, tests
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
line() {
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'order %.2f' % p['order_ms'], {x: round(k[x]['ms'],3) for x in ('cts_median',)})" $1 $2
}
for c in c3 c2; do
  for v in 0 1 0 1; do
    HGX_CTS_PAIR=$v timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b21_${c}_$v.json 2> $O/b21_${c}_$v.log || exit $?
    line $O/b21_${c}_$v.json ${c}_pair$v
  done
done
timeout -k 10 1100 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_incremental.py tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > $O/b21_tests.log 2>&1 || { tail -40 $O/b21_tests.log; exit 1; }
tail -1 $O/b21_tests.log
