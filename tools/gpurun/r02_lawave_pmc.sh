# SQ instruction counters of the lastAncestors kernels (16 time segments, c3 shape)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pmc_s && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d /tmp/pmc_s -o run -- python3 tools/probe/la_segs.py 256 10000000 16 > gpurun_out/pmc_s.log 2>&1 && \
python3 tools/rocpd_export.py counters /tmp/pmc_s/run_results.db gpurun_out/pmc_lawave_counters.csv
