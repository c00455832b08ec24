# host clock vs HIP events vs rocprofv3 for the same kernel windows (c3, c5)
set -o pipefail
mkdir -p gpurun_out/r05evt
O=gpurun_out/r05evt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c3 c5; do
  rm -rf /tmp/pe_$c
  HGX_HOST_TIME_KERNELS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pe_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/host_$c.log 2>&1 || exit 1
  python3 tools/rocpd_export.py stats /tmp/pe_$c/run_results.db $O/host_${c}_stats.csv || exit 1
  grep -c "host-timed" $O/host_$c.log
done
