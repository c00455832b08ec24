# two PMC passes (FETCH_SIZE, WRITE_SIZE) over one consensus pass of a config -> traffic json
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=${CFG:-c3}
# no warm-up context (hgx_create runs a small DAG once per process): its calls would count in the
# per-kernel averages and the traffic of the pass
export HGX_NO_WARMUP=1
rm -rf /tmp/pmc_f /tmp/pmc_w
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmc_f -o run -- python3 tools/phase_timing.py $CFG 1 > gpurun_out/pmc_f.log 2>&1 && \
python3 tools/rocpd_export.py counters /tmp/pmc_f/run_results.db gpurun_out/pmc_fetch_counters.csv && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d /tmp/pmc_w -o run -- python3 tools/phase_timing.py $CFG 1 > gpurun_out/pmc_w.log 2>&1 && \
python3 tools/rocpd_export.py counters /tmp/pmc_w/run_results.db gpurun_out/pmc_write_counters.csv && \
python3 tools/pmc_pass.py gpurun_out/pmc_fetch_counters.csv gpurun_out/pmc_write_counters.csv gpurun_out/traffic_$CFG.json
