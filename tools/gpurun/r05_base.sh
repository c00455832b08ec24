# round-5 baseline on a fresh box: the round-recurrence tests, the c3/c2 bench lines and the
# persistent kernel's phase clocks (prof build), then a rocprofv3 kernel trace of c3
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests/test_gpu_round_p.py -x -q --timeout 120 --timeout-method thread > $O/base_tests.log 2>&1 || { tail -30 $O/base_tests.log; exit 1; }
tail -1 $O/base_tests.log
for c in c3 c2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
    > $O/base_$c.json 2> $O/base_$c.log || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'value %.1f M' % (d['value']/1e6), 'coords %.2f rounds %.2f fame %.2f order %.2f' % (p['coords_ms'], p['rounds_ms'], p['fame_ms'], p['order_ms']))" $O/base_$c.json $c
done
for c in c3 c2; do
  HGX_LIB=libhgx_prof.so timeout -k 10 300 python -u tools/phase_timing.py $c 2 > $O/base_ph_$c.log 2>&1 || exit $?
  grep "k_round_p clk" $O/base_ph_$c.log | tail -1
done
