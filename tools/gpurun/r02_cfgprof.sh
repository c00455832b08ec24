# rocprofv3 kernel statistics of the c2, c4 and c5 bench commands (one trace per config)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in c2 c4 c5; do
  rm -rf /tmp/prof_$cfg && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$cfg -o run -- python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > gpurun_out/prof_${cfg}_bench.log 2>&1 && \
  python3 tools/rocpd_export.py stats /tmp/prof_$cfg/run_results.db gpurun_out/prof_${cfg}_kernel_stats.csv || exit 1
done
