# round-6 evidence on one box, per config (CFGS, default every config): PMC traffic + VALU passes
# (copied into profiles/ on the box so each bench line carries them), the rocprofv3 kernel trace of the
# config's bench command, the bench line; everything lands in gpurun_out/r06f/
set -o pipefail
mkdir -p gpurun_out/r06f
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in ${CFGS:-c3 c1 c2 c4 c5}; do
    CFG=$c bash tools/gpurun/pmc_traffic.sh || exit 1
    CFG=$c bash tools/gpurun/pmc_valu.sh || exit 1
    cp gpurun_out/traffic_$c.json gpurun_out/valu_$c.json profiles/ || exit 1
    cp gpurun_out/traffic_$c.json gpurun_out/valu_$c.json gpurun_out/r06f/ || exit 1
    cp gpurun_out/pmc_fetch_counters.csv gpurun_out/r06f/${c}_pmc_fetch_counters.csv
    cp gpurun_out/pmc_write_counters.csv gpurun_out/r06f/${c}_pmc_write_counters.csv
    cp gpurun_out/pmc_valu_counters_$c.csv gpurun_out/pmc_valu_stats_$c.csv gpurun_out/r06f/
    rm -rf /tmp/prof_c
    # (no warm-up context: its calls would enter the per-kernel averages, 7 timed passes + 1 tiny call)
    HGX_NO_WARMUP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > gpurun_out/r06f/${c}_prof.log 2>&1 || exit 1
    python3 tools/rocpd_export.py stats /tmp/prof_c/run_results.db gpurun_out/r06f/${c}_kernel_stats.csv || exit 1
    if [ "$c" = "c3" ]; then
        timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06f/c3_bench.json 2> gpurun_out/r06f/c3_bench.err || exit 1
    else
        timeout -k 10 300 python3 -u bench.py --config $c --steps 5 --warmup 1 > gpurun_out/r06f/${c}_bench.json 2> gpurun_out/r06f/${c}_bench.err || exit 1
    fi
    echo "$c done: $(tail -c 300 gpurun_out/r06f/${c}_bench.json)"
done
