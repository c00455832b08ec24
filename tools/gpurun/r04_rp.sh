# round 4: persistent recurrence -- parity tests, per-round trace (prof build), A/B bench lines
# usage: bash tools/gpurun/r04_rp.sh TAG "c3 c2" [ab-lib-tag ...]   (TESTS=0 skips the tests)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-rp}; CFGS=${2:-c3 c2}; shift 2 || true
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_round_p.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests0.log 2>&1 && timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.log
fi
for c in $CFGS; do
  HGX_LIB=libhgx_prof.so timeout -k 10 200 python -u tools/probe/rp_trace.py $c > gpurun_out/${TAG}_trace_$c.log 2>&1 || exit $?
  grep -v "^\[hgx\] \(round phases\|k_round_k\)" gpurun_out/${TAG}_trace_$c.log | grep -v amdgpu.ids | tail -16
  for L in "" "$@"; do
    lib=libhgx${L:+_$L}.so
    HGX_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
      > gpurun_out/${TAG}_${c}_${L:-new}.json 2> gpurun_out/${TAG}_${c}_${L:-new}.log || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'value %.1f M' % (d['value']/1e6), 'coords %.2f rounds %.2f fame %.2f order %.2f' % (p['coords_ms'], p['rounds_ms'], p['fame_ms'], p['order_ms']), 'fallbacks', p.get('round_p_fallbacks'))" gpurun_out/${TAG}_${c}_${L:-new}.json $lib
  done
done
