# bucket sort with in-kernel tie order (wave per bucket up to 512 events): tests, c4/c3 lines; first-call
# probe; c4 layout / sort PMC traffic
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_seg.py -x -v --timeout 200 --timeout-method thread > $O/s2_sort_tests.log 2>&1 || { tail -40 $O/s2_sort_tests.log; exit 1; }
tail -1 $O/s2_sort_tests.log
for c in c4 c3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
    > $O/s2_$c.json 2> $O/s2_$c.log || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'order %.2f' % p['order_ms'], 'seg', p.get('sort_seg'), {x: round(k[x]['ms'],3) for x in ('layout','order_sort','cts_median')})" $O/s2_$c.json $c
done
timeout -k 10 200 python -u tools/probe/first_call.py c3 > $O/s2_first.log 2>&1 || { tail -20 $O/s2_first.log; exit 1; }
grep -v amdgpu.ids $O/s2_first.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/s2_pf -o c4 -- python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/s2_pf.log 2>&1 || { tail -20 $O/s2_pf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/s2_pw -o c4 -- python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/s2_pw.log 2>&1 || { tail -20 $O/s2_pw.log; exit 1; }
echo pmc done
