# bench lines for a list of configs: bash tools/gpurun/bench_cfgs.sh TAG "c3 c2" [extra bench args]
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}; CFGS=${2:-c3}; shift 2 || true
for c in $CFGS; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest "$@" \
    > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.log || exit $?
done
