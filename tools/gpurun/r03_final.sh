# round-3 evidence on one box: PMC traffic + VALU passes at c3 (copied into profiles/ on the box so
# the bench line reads them), the rocprofv3 kernel trace of the bench command, the default bench line
# and the other configs' lines
set -o pipefail
mkdir -p gpurun_out/r03f
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpurun/pmc_traffic.sh && bash tools/gpurun/pmc_valu.sh && \
cp gpurun_out/traffic_c3.json gpurun_out/valu_c3.json profiles/ && \
rm -rf /tmp/prof_k && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_k -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > gpurun_out/r03f/prof_bench.log 2>&1 && \
python3 tools/rocpd_export.py stats /tmp/prof_k/run_results.db gpurun_out/r03f/c3_kernel_stats.csv && \
timeout -k 10 400 python3 -u bench.py > gpurun_out/r03f/c3_bench.json 2> gpurun_out/r03f/c3_bench.err && \
for c in c1 c2 c4 c5; do timeout -k 10 240 python3 -u bench.py --config $c --steps 5 --warmup 1 > gpurun_out/r03f/$c.json 2> gpurun_out/r03f/$c.err || exit 1; done
