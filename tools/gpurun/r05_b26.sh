# packed structure columns (hgx_events_packed): tests, then c3 / c4 host-RAM step packed vs compact
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_insert_and_run.py tests/test_pack_columns.py -x -v --timeout 200 --timeout-method thread > $O/b26_tests.log 2>&1 || { tail -40 $O/b26_tests.log; exit 1; }
tail -1 $O/b26_tests.log
line() {
  python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['config']['phase_ms_last_step']; print(sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'value %.1f M' % (d['value']/1e6), 'hbm %.2f' % d['hbm_resident']['ms_per_step'], 'rounds %.2f' % p['rounds_ms'])" $1 $2
}
for c in c3 c4; do
  for v in packed compact packed compact; do
    timeout -k 10 300 python -u bench.py --config $c --columns $v --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-check --no-chunked > $O/b26_${c}_$v.json 2> $O/b26_${c}_$v.log || exit $?
    line $O/b26_${c}_$v.json ${c}_$v
  done
done
