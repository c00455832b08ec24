#!/bin/bash
# whole-graph round kernel: parity tests, c4/c1 bench lines, phase profile (prof build)
set -o pipefail
cd "$(dirname "$0")/../.."
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_round_g.py tests/test_gpu_round_p.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rg_tests.log 2>&1 || { tail -30 gpurun_out/rg_tests.log; exit 1; }
tail -2 gpurun_out/rg_tests.log
$T 200 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-ingest > gpurun_out/rg_c4.json 2> gpurun_out/rg_c4.err || exit 1
$T 200 python bench.py --config c1 --steps 20 --warmup 3 > gpurun_out/rg_c1.json 2> gpurun_out/rg_c1.err || exit 1
for c in c1 c4; do
  HGX_LIB=libhgx_prof.so $T 150 python bench.py --config $c --steps 2 --warmup 0 --no-cpu-baseline --no-chunked --no-ingest --no-check > gpurun_out/rgp_$c.json 2> gpurun_out/rgp_$c.err || exit 1
  grep "k_round_g" gpurun_out/rgp_$c.err | tail -1
done
