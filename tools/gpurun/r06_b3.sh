# round 6: the small-order rank sort (256 x 64 tiles): the tests that reach it, then c1's line and the
# chunked c3 schedule's per-call profile
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_sort_seg.py \
  tests/test_gpu_insert_and_run.py tests/test_gpu_reset.py -x -q --timeout 300 --timeout-method thread > $O/b3_tests.log 2>&1 \
  || { tail -40 $O/b3_tests.log; exit 1; }
tail -1 $O/b3_tests.log
timeout -k 10 300 python -u bench.py --config c1 --steps 50 --warmup 5 --no-ingest > $O/b3_c1.json 2> $O/b3_c1.log || { tail -20 $O/b3_c1.log; exit 1; }
python tools/r06_summary.py $O/b3_c1.json
timeout -k 10 300 python -u tools/probe/chunked_profile.py c3 3000 1000 300 > $O/b3_chunk_c3.log 2>&1 || { tail -10 $O/b3_chunk_c3.log; exit 1; }
grep -v amdgpu.ids $O/b3_chunk_c3.log
for v in "ROC_ACTIVE_WAIT_TIMEOUT=1000" "ROC_ACTIVE_WAIT_TIMEOUT=0"; do
  env $v timeout -k 10 300 python -u tools/probe/chunked_profile.py c3 3000 1000 300 > $O/b3_chunk_c3_$v.log 2>&1 || { tail -10 "$O/b3_chunk_c3_$v.log"; exit 1; }
  echo "== $v"; grep "host total\|host divide\|host insert\|host fame\|host order" "$O/b3_chunk_c3_$v.log"
done
