# k_round_pb debug build: rows, window and per-candidate K checked in-kernel (printf on mismatch)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
PYTHONPATH=. HGX_LIB=libhgx_exp_pbchk.so timeout -k 10 300 python -u tools/probe/pb_diff.py 384,16000,0.2 > $O/pbchk.log 2>&1 || { tail -30 $O/pbchk.log; exit 1; }
grep -c PBCHK $O/pbchk.log || true
grep -v PBCHK $O/pbchk.log | tail -12
grep PBCHK-WIN $O/pbchk.log | head -20 || true
grep PBCHK-ROW $O/pbchk.log | head -20 || true
grep "PBCHK " $O/pbchk.log | head -10 || true
