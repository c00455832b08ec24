# k_round_p phase clocks of wave 1 (a rebasing wave; HGX_PROF_T=64 build) at c3
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
HGX_LIB=libhgx_exp3.so timeout -k 10 300 python -u tools/phase_timing.py c3 2 > $O/b20_ph_c3_w1.log 2>&1 || { tail -20 $O/b20_ph_c3_w1.log; exit 1; }
grep -E "k_round_p clk" $O/b20_ph_c3_w1.log | tail -1
