# consensus-timestamp kernel A/B: parity on the default library, then bench phases per variant
# usage: bash tools/gpurun/r04_cts.sh TAG "c3 c2 c5" variant [variant ...]   ("" = libhgx.so)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-cts}; CFGS=${2:-c3}; shift 2 || true
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_incremental.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/${TAG}_tests.log
for c in $CFGS; do
  for L in "$@"; do
    lib=libhgx${L:+_$L}.so
    HGX_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
      > gpurun_out/${TAG}_${c}_${L:-new}.json 2> gpurun_out/${TAG}_${c}_${L:-new}.log || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; print(sys.argv[2], sys.argv[3], 'ms/step %.2f' % d['ms_per_step'], 'coords %.2f rounds %.2f fame %.2f order %.2f' % (p['coords_ms'], p['rounds_ms'], p['fame_ms'], p['order_ms']))" gpurun_out/${TAG}_${c}_${L:-new}.json $c $lib
    grep -o "kernel profile.*" gpurun_out/${TAG}_${c}_${L:-new}.log | cut -c1-400
  done
done
