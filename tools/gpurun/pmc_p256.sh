# one PMC pass (SQ_INSTS_VALU) with the kernel trace over the P-256 verify leg -> profiles-ready json
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pmc_p
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU --kernel-trace -d /tmp/pmc_p -o run -- python3 tools/probe/p256_pmc.py > gpurun_out/pmc_p256.log 2>&1 && \
python3 tools/rocpd_export.py counters /tmp/pmc_p/run_results.db gpurun_out/pmc_valu_counters_p256.csv && \
python3 tools/rocpd_export.py stats /tmp/pmc_p/run_results.db gpurun_out/pmc_valu_stats_p256.csv && \
python3 tools/pmc_valu.py gpurun_out/pmc_valu_counters_p256.csv gpurun_out/pmc_valu_stats_p256.csv gpurun_out/valu_p256.json
