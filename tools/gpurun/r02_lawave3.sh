# dataflow lastAncestors pass: parity, then a kernel trace of a c3 bench run
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_la_wave.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lawave_tests.log 2>&1 && \
rm -rf /tmp/prof_k && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_k -o run -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > gpurun_out/prof_bench.log 2>&1 && \
python3 tools/rocpd_export.py stats /tmp/prof_k/run_results.db gpurun_out/prof_kernel_stats.csv
