# round 5 batch 3: the big-n persistent recurrence (k_round_pb): its tests, the k_round_p tests
# (regression), c5 bench lines with and without it
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_round_pb.py -x -v --timeout 200 --timeout-method thread -k "not c5_prefix" > $O/b3_pb.log 2>&1 || { tail -40 $O/b3_pb.log; exit 1; }
tail -1 $O/b3_pb.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_round_p.py -x -q --timeout 120 --timeout-method thread > $O/b3_rp.log 2>&1 || { tail -30 $O/b3_rp.log; exit 1; }
tail -1 $O/b3_rp.log
for rk in auto auto-steps; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked --round-kernel $rk \
    > $O/b3_c5_$rk.json 2> $O/b3_c5_$rk.log || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; k=d['kernels_per_pass']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'coords %.2f rounds %.2f fame %.2f order %.2f' % (p['coords_ms'], p['rounds_ms'], p['fame_ms'], p['order_ms']), 'runs', p.get('round_p_runs'), 'fb', p.get('round_p_fallbacks'), {x: k[x]['ms'] for x in k if k[x]['ms'] > 0.3})" $O/b3_c5_$rk.json $rk
done
