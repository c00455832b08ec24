# round 6: firstDescendants chunk loop with two positions per lane: the tests that read FD, then an
# A/B of c5 / c3 / c4 lines against the previous build (libhgx_old.so), twice, interleaved
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_la_wave.py tests/test_gpu_incremental.py \
  tests/test_gpu_round_pb.py tests/test_gpu_full_config.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread \
  > $O/fd4_tests.log 2>&1 || { tail -40 $O/fd4_tests.log; exit 1; }
tail -1 $O/fd4_tests.log
for rep in 1 2; do
  for c in c5 c3 c4; do
    for L in libhgx_old.so libhgx.so; do
      HGX_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-ingest \
        --no-check --no-chunked > $O/fd4_${c}_${L}_$rep.json 2> $O/fd4_${c}_${L}_$rep.log || { tail -20 $O/fd4_${c}_${L}_$rep.log; exit 1; }
      echo "$rep $L $(python tools/r06_summary.py $O/fd4_${c}_${L}_$rep.json | cut -c1-330)"
    done
  done
done
