# k_round_pb candidate rows chunk-major with SGPR chunk bases (libhgx_exp1.so) against the current build:
# probe, c5 A/B, pb tests on the new build
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
line() {
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'rounds %.2f' % p['rounds_ms'], 'rp', p['round_p_runs'], p['round_p_fallbacks'], {x: round(k[x]['ms'],3) for x in ('round_search',)})" $1 $2
}
HGX_LIB=libhgx_exp1.so PYTHONPATH=. timeout -k 10 400 python -u tools/probe/pb_diff.py > $O/b17_diff.log 2>&1 || { tail -30 $O/b17_diff.log; exit 1; }
grep -c "mismatch=0" $O/b17_diff.log
for v in libhgx.so libhgx_exp1.so libhgx.so libhgx_exp1.so; do
  HGX_LIB=$v timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b17_c5_$v.json 2> $O/b17_c5_$v.log || exit $?
  line $O/b17_c5_$v.json c5_$v
done
HGX_LIB=libhgx_exp1.so timeout -k 10 900 python -u -m pytest tests/test_gpu_round_pb.py -x -q --timeout 200 --timeout-method thread > $O/b17_tests.log 2>&1 || { tail -40 $O/b17_tests.log; exit 1; }
tail -1 $O/b17_tests.log
