# lastAncestors time-segment count: c2 beyond 96, c3 again without the verify sweep
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/probe/la_segs_sweep.py c2 96 128 192 256 > $O/b29_c2.log 2>&1 || { tail -20 $O/b29_c2.log; exit 1; }
cat $O/b29_c2.log | grep segs
timeout -k 10 400 python -u tools/probe/la_segs_sweep.py c3 0 16 24 32 48 64 > $O/b29_c3.log 2>&1 || { tail -20 $O/b29_c3.log; exit 1; }
cat $O/b29_c3.log | grep segs
