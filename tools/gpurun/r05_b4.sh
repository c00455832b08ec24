# warm-up at creation (first-call probe), k_round_pb FDT prefetch (c5), staged layout A/B (c4, c3), then
# the whole GPU suite
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/probe/first_call.py c3 > $O/b4_first.log 2>&1 || { tail -20 $O/b4_first.log; exit 1; }
grep -v amdgpu.ids $O/b4_first.log
line() {
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'rounds %.2f order %.2f coords %.2f' % (p['rounds_ms'], p['order_ms'], p['coords_ms']), {x: round(k[x]['ms'],3) for x in ('layout','order_sort','round_search')})" $1 $2
}
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b4_c5.json 2> $O/b4_c5.log || exit $?
line $O/b4_c5.json c5
HGX_LIB=libhgx_prof.so timeout -k 10 300 python -u tools/phase_timing.py c5 2 > $O/b4_ph_c5.log 2>&1 || { tail -20 $O/b4_ph_c5.log; exit 1; }
grep -E "k_round_pb clk" $O/b4_ph_c5.log | tail -1
for c in c4 c3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b4_$c.json 2> $O/b4_$c.log || exit $?
  line $O/b4_$c.json $c
  HGX_LAYOUT_ROUND4=1 timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b4_${c}_r4.json 2> $O/b4_${c}_r4.log || exit $?
  line $O/b4_${c}_r4.json ${c}_layout_r4
done
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/b4_suite.log 2>&1 || { tail -40 $O/b4_suite.log; exit 1; }
tail -2 $O/b4_suite.log
