# A/B of library variants on one box: parity of the round recurrence (test_gpu_round_p.py) per variant,
# then c3 / c2 bench lines per variant, twice, interleaved. usage: bash tools/gpurun/r06_ab.sh TAG lib1.so lib2.so ...
set -o pipefail
TAG=$1; shift
O=gpurun_out/r06
mkdir -p $O
for L in "$@"; do
  HGX_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_round_p.py -x -q --timeout 120 --timeout-method thread \
    > $O/${TAG}_tests_$L.log 2>&1 || { tail -30 $O/${TAG}_tests_$L.log; exit 1; }
  echo "$L: $(tail -1 $O/${TAG}_tests_$L.log)"
done
for rep in 1 2; do
  for c in c3 c2; do
    for L in "$@"; do
      HGX_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-ingest \
        --no-check --no-chunked > $O/${TAG}_${c}_${L}_$rep.json 2> $O/${TAG}_${c}_${L}_$rep.log || { tail -20 $O/${TAG}_${c}_${L}_$rep.log; exit 1; }
      echo "$rep $L $(python tools/r06_summary.py $O/${TAG}_${c}_${L}_$rep.json)"
    done
  done
done
