set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/prof_c3 /tmp/pmc_fetch /tmp/pmc_write
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_c3 -o c3 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 && \
python3 tools/rocpd_export.py stats /tmp/prof_c3/c3_results.db gpurun_out/c3_kernel_stats.csv && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmc_fetch -o c3 -- python3 tools/phase_timing.py c3 1 > gpurun_out/pmc_fetch.log 2>&1 && \
python3 tools/rocpd_export.py counters /tmp/pmc_fetch/c3_results.db gpurun_out/c3_fetch_counter_collection.csv && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/pmc_write -o c3 -- python3 tools/phase_timing.py c3 1 > gpurun_out/pmc_write.log 2>&1 && \
python3 tools/rocpd_export.py counters /tmp/pmc_write/c3_results.db gpurun_out/c3_write_counter_collection.csv
