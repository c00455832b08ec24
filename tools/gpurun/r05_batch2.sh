# round 5 batch 2: the remaining lastAncestors tests, c4 / c3 lines, A/B of the precomputed publish
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_la_wave.py -x -v --timeout 300 --timeout-method thread -k "segments or batched or small" > $O/b2_tests.log 2>&1 || { tail -40 $O/b2_tests.log; exit 1; }
tail -1 $O/b2_tests.log
for c in c4 c3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
    > $O/b2_$c.json 2> $O/b2_$c.log || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'la_verify', p.get('la_verify'), {x: k[x]['ms'] for x in ('layout','order_sort','round_search','la_sweep')})" $O/b2_$c.json $c
done
bash tools/gpurun/r04_ab.sh r05ab4 "c3 c2 c3 c2" "" exp_pub
