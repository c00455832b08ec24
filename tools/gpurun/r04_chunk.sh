#!/bin/bash
# chunked schedule at c3: per-call host/device breakdown, then a kernel trace of the same calls
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04c
timeout -k 10 300 python3 tools/probe/chunked_profile.py c3 700 1000 100 > gpurun_out/r04c/chunk_c3.log 2>&1 || exit 1
cat gpurun_out/r04c/chunk_c3.log | grep -v amdgpu.ids
rm -rf /tmp/prof_ch
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d /tmp/prof_ch -o run -- python3 tools/probe/chunked_profile.py c3 700 1000 100 > gpurun_out/r04c/chunk_prof.log 2>&1 || exit 1
python3 tools/rocpd_export.py stats /tmp/prof_ch/run_results.db gpurun_out/r04c/chunk_c3_kernel_stats.csv || exit 1
python3 tools/rocpd_export.py trace /tmp/prof_ch/run_results.db gpurun_out/r04c/chunk_trace.csv || exit 1
