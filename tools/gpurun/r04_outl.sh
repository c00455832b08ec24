#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
T="timeout -k 10"
mkdir -p gpurun_out/r04c
$T 500 python -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_round_p.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > gpurun_out/outl_tests.log 2>&1 || { tail -30 gpurun_out/outl_tests.log; exit 1; }
tail -2 gpurun_out/outl_tests.log
$T 300 python3 tools/probe/chunked_outliers.py c5 1100 2 > gpurun_out/r04c/outliers_c5.log 2>&1 || exit 1
tail -6 gpurun_out/r04c/outliers_c5.log
$T 300 python3 tools/probe/chunked_outliers.py c2 1100 1 > gpurun_out/r04c/outliers_c2.log 2>&1 || exit 1
tail -6 gpurun_out/r04c/outliers_c2.log
