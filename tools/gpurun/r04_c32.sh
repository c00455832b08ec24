set -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 ./tools/probe/h2d_bw > gpurun_out/h2d_bw.log 2>&1; cat gpurun_out/h2d_bw.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_insert_and_run.py tests/test_gpu_checkpoint.py tests/test_gpu_reset.py -x -q --timeout 150 --timeout-method thread > gpurun_out/c32_tests.log 2>&1 || { tail -30 gpurun_out/c32_tests.log; exit 1; }
tail -1 gpurun_out/c32_tests.log
for c in c3 c4; do for w in "" "--wide"; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked $w > gpurun_out/c32_${c}${w}.json 2> gpurun_out/c32_${c}${w}.log || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], 'ms/step %.2f' % d['ms_per_step'], 'value %.1f M' % (d['value']/1e6), 'hbm-resident %.2f ms' % d['hbm_resident']['ms_per_step'])" gpurun_out/c32_${c}${w}.json
done; done
bash tools/gpurun/r04_ab.sh ab3 "c3 c2" "" exppr exppg exppe
