# round-end evidence: all GPU tests, c3 bench line (with ingest leg), kernel stats of both
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/prof_f /tmp/prof_sha
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_sha -o sha -- python3 -c "import bench, json; print(json.dumps(bench.ingest_leg(10_000_000, 5, 2, 0)))" > gpurun_out/prof_sha.log 2>&1 && \
python3 tools/rocpd_export.py stats /tmp/prof_sha/sha_results.db gpurun_out/sha_kernel_stats.csv
