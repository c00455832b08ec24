# A/B of one environment switch on the default library: bench phases per setting
# usage: bash tools/gpurun/r04_env_ab.sh TAG "c3 c5" VAR "v1 v2 ..."
set -o pipefail
mkdir -p gpurun_out
TAG=$1; CFGS=$2; VAR=$3; VALS=$4
for c in $CFGS; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked \
      > gpurun_out/${TAG}_${c}_$v.json 2> gpurun_out/${TAG}_${c}_$v.log || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; print(sys.argv[2], sys.argv[3], 'ms/step %.2f' % d['ms_per_step'], 'coords %.2f rounds %.2f fame %.2f order %.2f' % (p['coords_ms'], p['rounds_ms'], p['fame_ms'], p['order_ms']))" gpurun_out/${TAG}_${c}_$v.json $c $VAR=$v
    grep -o "kernel profile.*" gpurun_out/${TAG}_${c}_$v.log | cut -c1-300
  done
done
