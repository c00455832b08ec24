# k_round_pb phase clocks of the window rebase (two row sets / one)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
for v in libhgx_prof.so libhgx_exp3.so; do
  HGX_LIB=$v timeout -k 10 300 python -u tools/phase_timing.py c5 2 > $O/b10_ph_$v.log 2>&1 || { tail -20 $O/b10_ph_$v.log; exit 1; }
  grep -E "k_round_pb clk" $O/b10_ph_$v.log | tail -1
done
