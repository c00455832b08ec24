# one PMC pass (SQ_INSTS_VALU) with the kernel trace over one consensus pass of a config -> valu json
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=${CFG:-c3}
# no warm-up context (hgx_create runs a small DAG once per process): its calls would count in the
# per-kernel averages and the traffic of the pass
export HGX_NO_WARMUP=1
rm -rf /tmp/pmc_v
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU --kernel-trace -d /tmp/pmc_v -o run -- python3 tools/phase_timing.py $CFG 1 > gpurun_out/pmc_v.log 2>&1 && \
python3 tools/rocpd_export.py counters /tmp/pmc_v/run_results.db gpurun_out/pmc_valu_counters_$CFG.csv && \
python3 tools/rocpd_export.py stats /tmp/pmc_v/run_results.db gpurun_out/pmc_valu_stats_$CFG.csv && \
python3 tools/pmc_valu.py gpurun_out/pmc_valu_counters_$CFG.csv gpurun_out/pmc_valu_stats_$CFG.csv gpurun_out/valu_$CFG.json
