# round 6, first box: the new sharded / launcher / packed / full-config tests, then c3 lines (one GPU,
# and --gpus 2 without a launcher: replicas + the chain-sharded leg, two shards on the one GPU)
set -o pipefail
mkdir -p gpurun_out/r06
O=gpurun_out/r06
timeout -k 10 1000 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_bench_dist.py tests/test_gpu_insert_and_run.py \
  tests/test_gpu_full_config.py tests/test_gpu_full_digests.py tests/test_gpu_sort_seg.py -x -v --timeout 300 --timeout-method thread > $O/b1_tests.log 2>&1 \
  || { tail -60 $O/b1_tests.log; exit 1; }
tail -1 $O/b1_tests.log
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline --no-ingest --no-chunked \
  > $O/b1_c3.json 2> $O/b1_c3.log || { tail -30 $O/b1_c3.log; exit 1; }
python tools/r06_summary.py $O/b1_c3.json
timeout -k 10 600 python -u bench.py --gpus 2 --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-chunked \
  > $O/b1_c3_g2.json 2> $O/b1_c3_g2.log || { tail -30 $O/b1_c3_g2.log; exit 1; }
python tools/r06_summary.py $O/b1_c3_g2.json
