# round 5: the chain-sharded group (every shard on device 0) and the round-recurrence / checkpoint
# suites, then c3 / c2 bench lines on the current build
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_round_p.py tests/test_gpu_checkpoint.py -x -v --timeout 300 --timeout-method thread > $O/shard_tests.log 2>&1 || { tail -40 $O/shard_tests.log; exit 1; }
tail -1 $O/shard_tests.log
for c in c3 c2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
    > $O/shard_$c.json 2> $O/shard_$c.log || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'value %.1f M' % (d['value']/1e6), 'coords %.2f rounds %.2f fame %.2f order %.2f' % (p['coords_ms'], p['rounds_ms'], p['fame_ms'], p['order_ms']))" $O/shard_$c.json $c
done
# the layout change at c4 (PMC-free timing from the bench line's kernel table)
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
  > $O/shard_c4.json 2> $O/shard_c4.log || exit $?
python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; print('c4 ms/step %.2f' % d['ms_per_step'], {x: k[x]['ms'] for x in ('layout','order_sort','round_search','la_sweep')})" $O/shard_c4.json
