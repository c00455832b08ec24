# k_round_pb 63-probe windows + add-based SWAR count in k_round_p / k_round_pb; A/B against the
# previous commit (libhgx_base.so), exp1 = one row set, exp2 = 31-probe windows; phases; round tests
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
line() {
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'rounds %.2f order %.2f coords %.2f' % (p['rounds_ms'], p['order_ms'], p['coords_ms']), 'rp', p['round_p_runs'], p['round_p_fallbacks'], {x: round(k[x]['ms'],3) for x in ('layout','order_sort','round_search')})" $1 $2
}
PYTHONPATH=. timeout -k 10 400 python -u tools/probe/pb_diff.py > $O/b9_diff.log 2>&1 || { tail -30 $O/b9_diff.log; exit 1; }
grep -c "mismatch=0" $O/b9_diff.log
for c in c5 c3 c2; do
  for v in libhgx_base.so libhgx.so libhgx_exp2.so libhgx_base.so libhgx.so; do
    HGX_LIB=$v timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b9_${c}_$v.json 2> $O/b9_${c}_$v.log || exit $?
    line $O/b9_${c}_$v.json ${c}_$v
  done
done
HGX_LIB=libhgx_exp1.so timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b9_c5_exp1.json 2> $O/b9_c5_exp1.log || exit $?
line $O/b9_c5_exp1.json c5_exp1
for c in c5 c3; do
  HGX_LIB=libhgx_prof.so timeout -k 10 300 python -u tools/phase_timing.py $c 2 > $O/b9_ph_$c.log 2>&1 || { tail -20 $O/b9_ph_$c.log; exit 1; }
  grep -E "k_round_pb? clk" $O/b9_ph_$c.log | tail -2
done
timeout -k 10 1100 python -u -m pytest tests/test_gpu_round_pb.py tests/test_gpu_round_p.py tests/test_gpu_sharded.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/b9_tests.log 2>&1 || { tail -40 $O/b9_tests.log; exit 1; }
tail -1 $O/b9_tests.log
