#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_insert_and_run.py tests/test_gpu_checkpoint.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pay_tests.log 2>&1 || { tail -30 gpurun_out/pay_tests.log; exit 1; }
tail -2 gpurun_out/pay_tests.log
for c in c4 c3; do
  $T 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/pay_$c.json 2> gpurun_out/pay_$c.err || exit 1
  python - $c <<'PY'
import json, sys
c = sys.argv[1]
d = json.load(open(f'gpurun_out/pay_{c}.json'))
print(c, 'host-RAM', round(d['ms_per_step'], 2), 'hbm', round(d['hbm_resident']['ms_per_step'], 2))
PY
done
