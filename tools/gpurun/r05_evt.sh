# HIP-event kernel times (events without / with the system fence) against rocprofv3's kernel durations
set -o pipefail
mkdir -p gpurun_out/r05evt
O=gpurun_out/r05evt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pe1 /tmp/pe2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pe1 -o run -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/nofence.log 2>&1 || exit 1
python3 tools/rocpd_export.py stats /tmp/pe1/run_results.db $O/nofence_stats.csv || exit 1
HGX_EVENT_SYSFENCE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pe2 -o run -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/fence.log 2>&1 || exit 1
python3 tools/rocpd_export.py stats /tmp/pe2/run_results.db $O/fence_stats.csv || exit 1
grep -h "kernel profile" $O/nofence.log $O/fence.log
