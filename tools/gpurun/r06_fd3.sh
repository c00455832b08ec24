# round 6: firstDescendants with two tile rows per lane (128-row tiles of 128 targets, HGX_FD_RPL=2)
# against one (64-row tiles of 256): the FD readers' tests under RPL=2, then c3 / c5 / c4 lines, twice
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
HGX_FD_RPL=4 timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_la_wave.py tests/test_gpu_incremental.py \
  tests/test_gpu_full_config.py -x -q --timeout 300 --timeout-method thread > $O/fd3_tests.log 2>&1 || { tail -40 $O/fd3_tests.log; exit 1; }
tail -1 $O/fd3_tests.log
for rep in 1 2; do
  for c in c3 c5 c4; do
    for R in 2 4; do
      HGX_FD_RPL=$R timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-ingest \
        --no-check --no-chunked > $O/fd3_${c}_${R}_$rep.json 2> $O/fd3_${c}_${R}_$rep.log || { tail -20 $O/fd3_${c}_${R}_$rep.log; exit 1; }
      python -c "import json; d=json.loads([l for l in open('$O/fd3_${c}_${R}_$rep.json') if l.startswith('{')][-1]); k=d['kernels_per_pass']; print('$rep RPL=$R $c', round(d['ms_per_step'],3), 'fd_build', round(k['fd_build']['ms'],3))"
    done
  done
done
