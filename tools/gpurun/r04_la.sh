#!/bin/bash
# small-graph lastAncestors: LA tests, c1 bench
set -o pipefail
cd "$(dirname "$0")/../.."
T="timeout -k 10"
$T 500 python -u -m pytest tests/test_gpu_la_wave.py tests/test_gpu_incremental.py -x -q --timeout 150 --timeout-method thread > gpurun_out/la_tests.log 2>&1 || { tail -30 gpurun_out/la_tests.log; exit 1; }
tail -2 gpurun_out/la_tests.log
$T 200 python bench.py --config c1 --steps 20 --warmup 3 > gpurun_out/la_c1.json 2> gpurun_out/la_c1.err || exit 1
python - <<'PY'
import json
d=json.load(open('gpurun_out/la_c1.json'))
print('c1', round(d['value']), round(d['ms_per_step'],3), {k:v for k,v in d['config']['phase_ms_last_step'].items() if k.endswith('_ms')})
print(' la', d['kernels_per_pass']['la_sweep'], 'cpu', d['cpu_baseline']['value'], 'chunked', d['chunked_sync']['ms_per_call'], d['chunked_sync']['worst_call_ms'])
PY
