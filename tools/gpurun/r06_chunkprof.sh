# round 6 (final build): the SyncLimit-chunked schedule per API call at c3 (host wall time per call and the
# device phase times), then the rocprofv3 kernel statistics of 1 000 such calls
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/probe/chunked_profile.py c3 3000 1000 300 > $O/chunk_c3.log 2>&1 || { tail -10 $O/chunk_c3.log; exit 1; }
grep -v amdgpu.ids $O/chunk_c3.log
rm -rf /tmp/pc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pc -o run -- python3 tools/probe/chunked_profile.py c3 1000 1000 100 > $O/chunk_prof.log 2>&1 || { tail -10 $O/chunk_prof.log; exit 1; }
python3 tools/rocpd_export.py stats /tmp/pc/run_results.db $O/chunk_kernel_stats.csv || exit 1
head -30 $O/chunk_kernel_stats.csv | cut -c1-150
