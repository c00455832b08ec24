# round 6 evidence: c3 host columns pageable vs page-locked (with the chunked leg's outliers), the
# one-GPU chain-sharded c3 rehearsals W = 2/4/8 (local and remote windows), and DecideFame's
# popcount vs int8-MFMA tally at c5 (timing + PMC)
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in; do
  HGX_XCHG_MODE=$m timeout -k 10 120 python -u tools/probe/xchg.py 2000 > $O/ev_xchg_$m.log 2>&1 || { tail -10 $O/ev_xchg_$m.log; exit 1; }
  grep -v amdgpu.ids $O/ev_xchg_$m.log
done
for hm in; do
  timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-ingest --no-check \
    --host-memory $hm > $O/ev_c3_$hm.json 2> $O/ev_c3_$hm.log || { tail -20 $O/ev_c3_$hm.log; exit 1; }
  echo "$hm $(python tools/r06_summary.py $O/ev_c3_$hm.json)"
  python -c "import json,sys; d=json.loads([l for l in open('$O/ev_c3_$hm.json') if l.startswith('{')][-1]); c=d.get('chunked_sync',{}); print({k:c.get(k) for k in ('ms_per_call','worst_call_ms','p99_call_ms','worst_calls')})"
done
for spec in "8 0" "8 1"; do
  set -- $spec
  R=""; [ "$2" = 1 ] && R="--remote-windows"
  timeout -k 10 400 python -u bench.py --sharded --gpus $1 --config ${SHCFG:-c2} --steps 3 --warmup 1 --no-cpu-baseline --no-check $R \
    > $O/ev_sh_w$1_r$2.json 2> $O/ev_sh_w$1_r$2.log || { tail -20 $O/ev_sh_w$1_r$2.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/ev_sh_w$1_r$2.json') if l.startswith('{')][-1]); p=d['config']['phase_ms_last_step']; print('W=$1 remote=$2', round(d['ms_per_step'],2), 'ms', round(d['value']/1e6,1), 'M/s rounds', p['rounds_ms'], 'fallbacks', p['round_p_fallbacks'], d['config']['windows'])"
done
export HGX_NO_WARMUP=1
for t in popc mfma; do
  HGX_FAME_TALLY=$t timeout -k 10 200 python -u tools/phase_timing.py c5 3 > $O/ev_fame_$t.log 2>&1 || { tail -10 $O/ev_fame_$t.log; exit 1; }
  tail -1 $O/ev_fame_$t.log | cut -c1-200
  rm -rf /tmp/pmc_f
  HGX_FAME_TALLY=$t timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace \
    -d /tmp/pmc_f -o run -- python3 tools/phase_timing.py c5 1 > $O/ev_fame_pmc_$t.log 2>&1 || { tail -10 $O/ev_fame_pmc_$t.log; exit 1; }
  python3 tools/rocpd_export.py counters /tmp/pmc_f/run_results.db $O/ev_fame_pmc_counters_$t.csv || exit 1
  grep -i "fame" $O/ev_fame_pmc_counters_$t.csv | head -8
done
timeout -k 10 300 python -u tools/probe/chunked_profile.py c3 3000 1000 300 > $O/ev_chunk_c3.log 2>&1 || { tail -10 $O/ev_chunk_c3.log; exit 1; }
grep -v amdgpu.ids $O/ev_chunk_c3.log
rm -rf /tmp/pc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pc -o run -- python3 tools/probe/chunked_profile.py c3 1000 1000 100 > $O/ev_chunk_prof.log 2>&1 || { tail -10 $O/ev_chunk_prof.log; exit 1; }
python3 tools/rocpd_export.py stats /tmp/pc/run_results.db $O/ev_chunk_stats.csv || exit 1
head -30 $O/ev_chunk_stats.csv | cut -c1-150
