# round 6: round received with ballot slots and 4 events per thread, the witness-row transpose in 16-byte
# tiles, the post pass's compact WLA copy two coordinates per lane, the thresholds' k-th value by bisection on
# ballots: the whole GPU suite and smoke, an A/B of c3 / c2 / c4 lines against the previous build
# (libhgx_old.so), and the rocprofv3 kernel statistics of the new build at c3
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=rr bash tools/gpurun/r06_suite.sh || exit 1
for c in c3 c2 c4; do
  for L in libhgx_old.so libhgx.so; do
    HGX_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-ingest \
      --no-check --no-chunked > $O/rr_${c}_${L}.json 2> $O/rr_${c}_${L}.log || { tail -20 $O/rr_${c}_${L}.log; exit 1; }
    echo "$L $(python tools/r06_summary.py $O/rr_${c}_${L}.json | cut -c1-700)"
  done
done
rm -rf /tmp/prof_c
HGX_NO_WARMUP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_c -o run -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/rr_c3_prof.log 2>&1 || exit 1
python3 tools/rocpd_export.py stats /tmp/prof_c/run_results.db $O/rr_c3_kernel_stats.csv || exit 1
grep -E "threshold|transpose|round_received|round_p_post" $O/rr_c3_kernel_stats.csv | cut -c1-160
