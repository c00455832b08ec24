# one PMC pass over the ingest kernel (VALU issue vs busy cycles)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pmc_sha
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d /tmp/pmc_sha -o sha -- python3 -c "from babble_amd.hashgraph import sha256_bench as b; print(b(10_000_000, 400, 560, 5, warmup=0, iters=1, n_sample=1)['ms_per_launch'])" > gpurun_out/pmc_sha.log 2>&1 && \
python3 tools/rocpd_export.py counters /tmp/pmc_sha/sha_results.db gpurun_out/sha_pmc_counters.csv
