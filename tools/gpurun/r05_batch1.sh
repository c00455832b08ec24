# round 5 batch: sharded-group + round_p + checkpoint + lastAncestors suites on the current build, then
# c3 / c2 / c4 lines and an A/B of the precomputed-publish variant (libhgx_exp_pub.so)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_round_p.py tests/test_gpu_checkpoint.py tests/test_gpu_la_wave.py -x -v --timeout 300 --timeout-method thread > $O/b1_tests.log 2>&1 || { tail -40 $O/b1_tests.log; exit 1; }
tail -1 $O/b1_tests.log
for c in c4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
    > $O/b1_$c.json 2> $O/b1_$c.log || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; print('c4 ms/step %.2f' % d['ms_per_step'], {x: k[x]['ms'] for x in ('layout','order_sort','round_search','la_sweep')})" $O/b1_$c.json
done
bash tools/gpurun/r04_ab.sh r05ab4 "c3 c2 c3 c2" "" exp_pub
