# k_round_p wave priorities: HEAD vs exp1 (no priority for the younger half's search) vs exp2 (no top
# priority during the poll), c3
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
line() {
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'rounds %.2f' % p['rounds_ms'], {x: round(k[x]['ms'],3) for x in ('round_search',)})" $1 $2
}
for v in libhgx.so libhgx_exp1.so libhgx_exp2.so libhgx.so libhgx_exp1.so libhgx_exp2.so; do
  HGX_LIB=$v timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b25_c3_$v.json 2> $O/b25_c3_$v.log || exit $?
  line $O/b25_c3_$v.json c3_$v
done
