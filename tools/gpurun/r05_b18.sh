# k_round_p phase clocks with the publish phase split (prof build), c3 and c2
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
for c in c3 c2; do
  HGX_LIB=libhgx_prof.so timeout -k 10 300 python -u tools/phase_timing.py $c 2 > $O/b18_ph_$c.log 2>&1 || { tail -20 $O/b18_ph_$c.log; exit 1; }
  grep -E "k_round_p clk" $O/b18_ph_$c.log | tail -1
done
