# chunked-schedule A/B: incremental-path tests on the default library, then the c3 bench line's
# chunked leg (10 000 calls of 1 000 events) per library variant
# usage: bash tools/gpurun/r04_chunk_ab.sh TAG "c3" variant [variant ...]   ("" = libhgx.so)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-chab}; CFGS=${2:-c3}; shift 2 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for c in $CFGS; do
  for L in "$@"; do
    lib=libhgx${L:+_$L}.so
    HGX_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-check \
      > gpurun_out/${TAG}_${c}_${L:-new}.json 2> gpurun_out/${TAG}_${c}_${L:-new}.log || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); ch=d['config'].get('chunked_sync') or d.get('chunked_sync'); print(sys.argv[2], sys.argv[3], 'ms/step %.2f' % d['ms_per_step'], 'chunked ms/call %.4f worst %.3f' % (ch['ms_per_call'], ch['worst_call_ms']))" gpurun_out/${TAG}_${c}_${L:-new}.json $c $lib
  done
done
