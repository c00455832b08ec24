# lastAncestors time-segment count at c2 and c5 (coordinates phase of a full DivideRounds)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/probe/la_segs_sweep.py c2 0 16 24 32 48 64 96 > $O/b28_c2.log 2>&1 || { tail -20 $O/b28_c2.log; exit 1; }
cat $O/b28_c2.log | grep segs
timeout -k 10 300 python -u tools/probe/la_segs_sweep.py c5 0 2 4 8 > $O/b28_c5.log 2>&1 || { tail -20 $O/b28_c5.log; exit 1; }
cat $O/b28_c5.log | grep segs
