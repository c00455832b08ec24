set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/prof_l && \
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_l -o run -- python3 tools/probe/la_segs.py 256 10000000 16,32 > gpurun_out/la_segs_prof.log 2>&1 && \
python3 tools/rocpd_export.py trace /tmp/prof_l/run_results.db gpurun_out/la_trace.csv 'la_|fill|fd_build|layout'
