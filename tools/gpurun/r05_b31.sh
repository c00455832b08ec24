# the default build after the segment-cap flip: smoke, lastAncestors + full-workload tests, c2 line
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/b31_smoke.log 2>&1 || { tail -20 $O/b31_smoke.log; exit 1; }
tail -2 $O/b31_smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_la_wave.py tests/test_gpu_full_config.py -x -q --timeout 400 --timeout-method thread > $O/b31_tests.log 2>&1 || { tail -40 $O/b31_tests.log; exit 1; }
tail -1 $O/b31_tests.log
timeout -k 10 300 python -u bench.py --config c2 --steps 5 --warmup 1 > $O/b31_c2.json 2> $O/b31_c2.log || exit 1
python -c "import json; d=json.load(open('$O/b31_c2.json')); print(d['value']/1e6, d['ms_per_step'], d['config']['phase_ms_last_step'])"
