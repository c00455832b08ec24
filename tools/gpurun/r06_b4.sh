# round 6: bucket-sort tables sized for the round capacity (no reallocation inside a chunked FindOrder):
# the tests through the bucket sort, then the whole c3 chunked schedule's per-call profile
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_seg.py tests/test_gpu_incremental.py tests/test_gpu_full_config.py \
  -x -q --timeout 300 --timeout-method thread > $O/b4_tests.log 2>&1 || { tail -40 $O/b4_tests.log; exit 1; }
tail -1 $O/b4_tests.log
timeout -k 10 300 python -u tools/probe/chunked_profile.py c3 10000 1000 0 > $O/b4_chunk_c3.log 2>&1 || { tail -10 $O/b4_chunk_c3.log; exit 1; }
grep -v amdgpu.ids $O/b4_chunk_c3.log
