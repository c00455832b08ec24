# round-4 evidence for the other configs: PMC traffic + VALU per config (copied into profiles/ on the
# box so each bench line carries them), the rocprofv3 kernel trace of each config's bench command, and
# the bench lines
set -o pipefail
mkdir -p gpurun_out/r04c
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in ${CFGS:-c1 c2 c4 c5}; do
    CFG=$c bash tools/gpurun/pmc_traffic.sh || exit 1
    CFG=$c bash tools/gpurun/pmc_valu.sh || exit 1
    cp gpurun_out/traffic_$c.json gpurun_out/valu_$c.json profiles/ || exit 1
    cp gpurun_out/pmc_fetch_counters.csv gpurun_out/r04c/${c}_pmc_fetch_counters.csv
    cp gpurun_out/pmc_write_counters.csv gpurun_out/r04c/${c}_pmc_write_counters.csv
    cp gpurun_out/pmc_valu_counters_$c.csv gpurun_out/pmc_valu_stats_$c.csv gpurun_out/r04c/
    rm -rf /tmp/prof_c
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > gpurun_out/r04c/${c}_prof.log 2>&1 || exit 1
    python3 tools/rocpd_export.py stats /tmp/prof_c/run_results.db gpurun_out/r04c/${c}_kernel_stats.csv || exit 1
    timeout -k 10 240 python3 -u bench.py --config $c --steps 5 --warmup 1 > gpurun_out/r04c/$c.json 2> gpurun_out/r04c/$c.err || exit 1
    echo "$c done"
done
