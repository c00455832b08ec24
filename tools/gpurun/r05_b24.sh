# k_round_p: loop-invariant scalars and pointers laundered through empty asm (no kernel-argument
# rematerialisation; libhgx_exp1.so) against HEAD: A/B c2 c3, tests on the experiment build
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
line() {
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'rounds %.2f' % p['rounds_ms'], {x: round(k[x]['ms'],3) for x in ('round_search',)})" $1 $2
}
for c in c2 c3; do
  for v in libhgx.so libhgx_exp1.so libhgx.so libhgx_exp1.so; do
    HGX_LIB=$v timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b24_${c}_$v.json 2> $O/b24_${c}_$v.log || exit $?
    line $O/b24_${c}_$v.json ${c}_$v
  done
done
HGX_LIB=libhgx_exp1.so timeout -k 10 900 python -u -m pytest tests/test_gpu_round_p.py tests/test_gpu_sharded.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/b24_tests.log 2>&1 || { tail -40 $O/b24_tests.log; exit 1; }
tail -1 $O/b24_tests.log
