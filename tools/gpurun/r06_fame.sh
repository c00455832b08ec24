# round 6: DecideFame's tally re-measured on the current k_fame_tile: popcount against the
# int8 MFMA tally at c5 (1 024 peers, 341 silent) and c3, one PMC pass of 8 SQ counters over one consensus
# pass each, then the device phase times of the same config without the profiler
set -o pipefail
O=gpurun_out/r06fame
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HGX_NO_WARMUP=1
CTR="SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES"
for c in c5 c3; do
  for t in popc mfma; do
    rm -rf /tmp/pmc_f
    HGX_FAME_TALLY=$t timeout -s KILL 200 rocprofv3 --pmc $CTR --kernel-trace -d /tmp/pmc_f -o run -- \
      python3 tools/phase_timing.py $c 1 > $O/${c}_${t}_pmc.log 2>&1 || { tail -20 $O/${c}_${t}_pmc.log; exit 1; }
    python3 tools/rocpd_export.py counters /tmp/pmc_f/run_results.db $O/${c}_${t}_counters.csv || exit 1
    python3 tools/rocpd_export.py stats /tmp/pmc_f/run_results.db $O/${c}_${t}_stats.csv || exit 1
    HGX_FAME_TALLY=$t timeout -k 10 200 python3 tools/phase_timing.py $c 3 > $O/${c}_${t}_phases.log 2>&1 \
      || { tail -20 $O/${c}_${t}_phases.log; exit 1; }
    tail -1 $O/${c}_${t}_phases.log | cut -c1-400
  done
done
python3 tools/fame_pmc.py $O profiles/r06_fame_pmc.json && cp profiles/r06_fame_pmc.json $O/
