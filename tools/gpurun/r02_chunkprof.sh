# kernel trace of the SyncLimit-chunked schedule (c3 shape, 1 M events, 1 000-event calls)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/prof_ch && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ch -o run -- python3 tools/probe/chunk_calls.py 256 1000000 1000 > gpurun_out/chunkprof.log 2>&1 && \
python3 tools/rocpd_export.py stats /tmp/prof_ch/run_results.db gpurun_out/chunk_kernel_stats.csv
