# c5 line (k_round_pb, publish gathers first) + rocprofv3 kernel stats of c4 and c3 (segmented sort, layout)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
    > $O/pf1_c5.json 2> $O/pf1_c5.log || exit $?
python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_per_pass']; p=d['config']['phase_ms_last_step']; print('c5 ms/step %.2f' % d['ms_per_step'], 'rounds %.2f' % p['rounds_ms'], 'rp', p['round_p_runs'], p['round_p_fallbacks'])" $O/pf1_c5.json
HGX_LIB=libhgx_prof.so timeout -k 10 300 python -u tools/phase_timing.py c5 2 > $O/pf1_ph_c5.log 2>&1 || { tail -20 $O/pf1_ph_c5.log; exit 1; }
grep -E "k_round_pb clk" $O/pf1_ph_c5.log | tail -1
for c in c4 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pf1_rp_$c -o $c -- python3 -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/pf1_rp_$c.log 2>&1 || { tail -20 $O/pf1_rp_$c.log; exit 1; }
  f=$(find $O/pf1_rp_$c -name "*kernel_stats.csv" | head -1)
  head -25 "$f" | cut -d, -f1-5
done
