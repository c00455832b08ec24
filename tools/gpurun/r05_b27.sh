# full-workload bit-exact parity (c2, c4) and the default bench line
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_config.py -v --timeout 400 --timeout-method thread > $O/b27_full_config.log 2>&1 || { tail -40 $O/b27_full_config.log; exit 1; }
tail -4 $O/b27_full_config.log
timeout -k 10 600 python -u bench.py > $O/b27_c3_bench.json 2> $O/b27_c3_bench.err || exit 1
python -c "import json; d=json.load(open('$O/b27_c3_bench.json')); print(d['value']/1e6, d['ms_per_step'], d['chunked_sync']['ms_per_call'], d['chunked_sync']['worst_call_ms'])"
