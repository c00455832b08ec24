#!/bin/bash
# comb-table P-256: vector tests, verified insert tests, the 1 M-signature leg
set -o pipefail
cd "$(dirname "$0")/../.."
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_p256.py tests/test_gpu_verify_insert.py -x -q --timeout 200 --timeout-method thread > gpurun_out/p256_tests.log 2>&1 || { tail -30 gpurun_out/p256_tests.log; exit 1; }
tail -2 gpurun_out/p256_tests.log
$T 200 python -c "
import json, sys, time
sys.path.insert(0, '.')
import bench
t = time.time()
r = bench.p256_leg(1 << 20, 10, 3, 0)
print(json.dumps({k: v for k, v in r.items() if k != 'roofline'}))
print('leg wall s', round(time.time() - t, 1))
" > gpurun_out/p256_leg.log 2>&1 || { tail -20 gpurun_out/p256_leg.log; exit 1; }
cat gpurun_out/p256_leg.log | grep -v amdgpu.ids
