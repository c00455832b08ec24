# round 6: b1 (tests + c3 lines) then the per-round trace of the persistent recurrence (prof build)
set -o pipefail
bash tools/gpurun/r06_b1.sh || exit $?
O=gpurun_out/r06
for c in c3 c2; do
  HGX_LIB=libhgx_prof.so timeout -k 10 300 python -u tools/probe/rp_trace.py $c > $O/b2_trace_$c.log 2>&1 || { tail -20 $O/b2_trace_$c.log; exit 1; }
  grep -v "k_round_k\|k_round_g\|round phases" $O/b2_trace_$c.log | tail -22
done
