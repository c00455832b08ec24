# round-4 evidence on one box: PMC traffic + VALU passes at c3 and the P-256 VALU pass (copied into
# profiles/ on the box so the bench line reads them), the rocprofv3 kernel trace of the bench
# command, the default bench line
set -o pipefail
mkdir -p gpurun_out/r04f
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpurun/pmc_traffic.sh && bash tools/gpurun/pmc_valu.sh && bash tools/gpurun/pmc_p256.sh && \
cp gpurun_out/traffic_c3.json gpurun_out/valu_c3.json gpurun_out/valu_p256.json profiles/ && \
cp gpurun_out/pmc_fetch_counters.csv gpurun_out/r04f/c3_pmc_fetch_counters.csv && \
cp gpurun_out/pmc_write_counters.csv gpurun_out/r04f/c3_pmc_write_counters.csv && \
rm -rf /tmp/prof_k && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_k -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > gpurun_out/r04f/prof_bench.log 2>&1 && \
python3 tools/rocpd_export.py stats /tmp/prof_k/run_results.db gpurun_out/r04f/c3_kernel_stats.csv && \
timeout -k 10 500 python3 -u bench.py > gpurun_out/r04f/c3_bench.json 2> gpurun_out/r04f/c3_bench.err && \
tail -c 600 gpurun_out/r04f/c3_bench.json
