# round 6: the bucket sort in four parts with each part's order copied to the host (DMA, second stream) while
# the next part sorts: the tests through the bucket sort and the order (full c2 / c3 / c4 / c5 pins
# included), then an A/B of c3 / c4 / c2 against the previous build (libhgx_pre.so), twice (c2 once)
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_sort_seg.py tests/test_gpu_full_config.py tests/test_gpu_full_digests.py \
  tests/test_gpu_scale.py tests/test_gpu_insert_and_run.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > $O/sp_tests.log 2>&1 || { tail -40 $O/sp_tests.log; exit 1; }
tail -1 $O/sp_tests.log
for rep in 1 2; do
  for c in c3 c4 $([ $rep = 1 ] && echo c2); do
    for L in libhgx_pre.so libhgx.so; do
      HGX_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-ingest \
        --no-check --no-chunked > $O/sp_${c}_${L}_$rep.json 2> $O/sp_${c}_${L}_$rep.log || { tail -20 $O/sp_${c}_${L}_$rep.log; exit 1; }
      echo "$rep $L $(python tools/r06_summary.py $O/sp_${c}_${L}_$rep.json | cut -c1-700)"
    done
  done
done
