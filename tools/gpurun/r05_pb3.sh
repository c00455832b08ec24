# k_round_pb with the conflict-free window layout: probe + tests + c5 line + phase clocks; first-call
# probe after a warm-up context; c3 kernel stats (bucket sort breakdown)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
PYTHONPATH=. timeout -k 10 400 python -u tools/probe/pb_diff.py > $O/pb3_diff.log 2>&1 || { tail -30 $O/pb3_diff.log; exit 1; }
grep -c "mismatch=0" $O/pb3_diff.log
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
    > $O/pb3_c5.json 2> $O/pb3_c5.log || exit $?
python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; print('c5 ms/step %.2f' % d['ms_per_step'], 'rounds %.2f' % p['rounds_ms'], 'rp', p['round_p_runs'], p['round_p_fallbacks'])" $O/pb3_c5.json
HGX_LIB=libhgx_prof.so timeout -k 10 300 python -u tools/phase_timing.py c5 2 > $O/pb3_ph_c5.log 2>&1 || { tail -20 $O/pb3_ph_c5.log; exit 1; }
grep -E "k_round_pb clk" $O/pb3_ph_c5.log | tail -1
timeout -k 10 200 python -u tools/probe/first_call.py c3 warm > $O/pb3_first.log 2>&1 || { tail -20 $O/pb3_first.log; exit 1; }
grep -v amdgpu.ids $O/pb3_first.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pb3_rp_c3 -o c3 -- python3 -u bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/pb3_rp_c3.log 2>&1 || { tail -20 $O/pb3_rp_c3.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_round_pb.py -x -q --timeout 200 --timeout-method thread > $O/pb3_tests.log 2>&1 || { tail -40 $O/pb3_tests.log; exit 1; }
tail -1 $O/pb3_tests.log
