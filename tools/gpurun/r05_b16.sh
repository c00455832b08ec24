# c4 with 8-byte S-prefix loads in the bucket sort (A/B); the chunked schedule at c3 per API call and
# its kernels (rocprofv3)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
line() {
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], {x: round(k[x]['ms'],3) for x in ('layout','order_sort')})" $1 $2
}
for v in libhgx_base.so libhgx.so libhgx_base.so libhgx.so; do
  HGX_LIB=$v timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b16_c4_$v.json 2> $O/b16_c4_$v.log || exit $?
  line $O/b16_c4_$v.json c4_$v
done
rm -rf /tmp/pch
HGX_NO_WARMUP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pch -o run -- python3 tools/probe/chunked_profile.py c3 2000 1000 200 > $O/b16_chunk_c3.log 2>&1 || { tail -20 $O/b16_chunk_c3.log; exit 1; }
python3 tools/rocpd_export.py stats /tmp/pch/run_results.db $O/b16_chunk_c3_stats.csv || exit 1
grep -E "host|device|worst" $O/b16_chunk_c3.log | head -20
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_seg.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/b16_tests.log 2>&1 || { tail -40 $O/b16_tests.log; exit 1; }
tail -1 $O/b16_tests.log
