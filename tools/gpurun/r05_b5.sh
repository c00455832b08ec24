# bucket sort with 1 024-thread workgroups (c3), k_round_pb publish order (c5), chunked-call kernel profile
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
line() {
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'rounds %.2f order %.2f coords %.2f' % (p['rounds_ms'], p['order_ms'], p['coords_ms']), {x: round(k[x]['ms'],3) for x in ('layout','order_sort','round_search')})" $1 $2
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_seg.py -x -q --timeout 200 --timeout-method thread > $O/b5_sort_tests.log 2>&1 || { tail -40 $O/b5_sort_tests.log; exit 1; }
tail -1 $O/b5_sort_tests.log
for c in c3 c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b5_$c.json 2> $O/b5_$c.log || exit $?
  line $O/b5_$c.json $c
done
HGX_LIB=libhgx_prof.so timeout -k 10 300 python -u tools/phase_timing.py c5 2 > $O/b5_ph_c5.log 2>&1 || { tail -20 $O/b5_ph_c5.log; exit 1; }
grep -E "k_round_pb clk" $O/b5_ph_c5.log | tail -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/b5_chunk -o ch -- python3 -u tools/probe/chunked_profile.py c3 400 1000 50 > $O/b5_chunk.log 2>&1 || { tail -20 $O/b5_chunk.log; exit 1; }
grep -v amdgpu $O/b5_chunk.log | head -12
