# c5: round-step phase clocks and the rocprofv3 kernel trace (per-launch durations)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HGX_LIB=libhgx_prof.so timeout -k 10 200 python -u tools/phase_timing.py c5 2 > gpurun_out/c5_phases.log 2>&1 && \
rm -rf /tmp/prof_c5 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_c5 -o run -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > gpurun_out/c5_prof_bench.log 2>&1 && \
python3 tools/rocpd_export.py trace /tmp/prof_c5/run_results.db gpurun_out/c5_round_trace.csv 'k_round_k|k_la_sweep|k_fd_build' && \
python3 tools/rocpd_export.py stats /tmp/prof_c5/run_results.db gpurun_out/c5_kernel_stats.csv
