#!/bin/bash
# chain-sharded recurrence rehearsal: tests, then c3 rounds with W = 1, 2, 4
set -o pipefail
cd "$(dirname "$0")/../.."
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 || { tail -30 gpurun_out/shard_tests.log; exit 1; }
tail -2 gpurun_out/shard_tests.log
for w in 1 2 4 8; do
  GPU_MAX_HW_QUEUES=12 $T 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-chunked --no-check --round-shards $w > gpurun_out/shard_c3_w$w.json 2> gpurun_out/shard_c3_w$w.err || exit 1
  python - $w <<'PY'
import json, sys
w = sys.argv[1]
d = json.load(open(f'gpurun_out/shard_c3_w{w}.json'))
ph = d['config']['phase_ms_last_step']
print('W', w, 'step', round(d['ms_per_step'], 2), 'rounds', ph['rounds_ms'], 'coords', ph['coords_ms'], 'runs', ph['round_p_runs'],
      'fallbacks', ph['round_p_fallbacks'], 'fd', d['kernels_per_pass']['fd_build']['ms'], 'search', d['kernels_per_pass']['round_search']['ms'])
PY
done
