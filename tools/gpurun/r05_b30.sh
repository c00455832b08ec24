# lastAncestors segments up to the CUs' capacity (c2 16 -> 128): tests, then c2 / c3 bench lines
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
HGX_LIB=libhgx_exp1.so timeout -k 10 900 python -u -m pytest tests/test_gpu_la_wave.py tests/test_gpu_full_config.py tests/test_gpu_parity.py tests/test_gpu_insert_and_run.py tests/test_gpu_scale.py -x -q --timeout 400 --timeout-method thread > $O/b30_tests.log 2>&1 || { tail -40 $O/b30_tests.log; exit 1; }
tail -1 $O/b30_tests.log
for c in c2 c3; do
  HGX_LIB=libhgx_exp1.so timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b30_${c}.json 2> $O/b30_${c}.log || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms %.2f' % d['ms_per_step'], 'value %.1f M' % (d['value']/1e6), 'coords', p['coords_ms'], 'segs', p['la_wave_segs'], 'verify', p.get('la_verify'))" $O/b30_${c}.json $c
done
