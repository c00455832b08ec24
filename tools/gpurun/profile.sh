# rocprofv3 kernel trace of the c3 bench and the two PMC traffic passes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/prof_k && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_k -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > gpurun_out/prof_bench.log 2>&1 && \
python3 tools/rocpd_export.py stats /tmp/prof_k/run_results.db gpurun_out/prof_kernel_stats.csv && \
bash tools/gpurun/pmc_traffic.sh
