# A/B of library variants: round_p parity tests on each variant, then bench lines
# usage: bash tools/gpurun/r04_ab.sh TAG "c3 c2" variant [variant ...]   ("" = libhgx.so)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-ab}; CFGS=${2:-c3}; shift 2 || true
for L in "$@"; do
  lib=libhgx${L:+_$L}.so
  HGX_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_round_p.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests_${L:-new}.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests_${L:-new}.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/${TAG}_tests_${L:-new}.log)"
done
for c in $CFGS; do
  for L in "$@"; do
    lib=libhgx${L:+_$L}.so
    HGX_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
      > gpurun_out/${TAG}_${c}_${L:-new}.json 2> gpurun_out/${TAG}_${c}_${L:-new}.log || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; print(sys.argv[2], sys.argv[3], 'ms/step %.2f' % d['ms_per_step'], 'value %.1f M' % (d['value']/1e6), 'coords %.2f rounds %.2f fame %.2f order %.2f' % (p['coords_ms'], p['rounds_ms'], p['fame_ms'], p['order_ms']), 'fallbacks', p.get('round_p_fallbacks'))" gpurun_out/${TAG}_${c}_${L:-new}.json $c $lib
  done
done
