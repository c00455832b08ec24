# k_round_pb debugging: pb vs steps over a grid of traces, then c5 bench lines with and without it
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
PYTHONPATH=. timeout -k 10 400 python -u tools/probe/pb_diff.py > $O/pbdbg.log 2>&1 || { tail -30 $O/pbdbg.log; exit 1; }
cat $O/pbdbg.log
for rk in auto auto-steps; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked --round-kernel $rk \
    > $O/pbdbg_c5_$rk.json 2> $O/pbdbg_c5_$rk.log || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; k=d['kernels_per_pass']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'coords %.2f rounds %.2f fame %.2f order %.2f' % (p['coords_ms'], p['rounds_ms'], p['fame_ms'], p['order_ms']), {x: k[x]['ms'] for x in k if k[x]['ms'] > 0.3})" $O/pbdbg_c5_$rk.json $rk
done
