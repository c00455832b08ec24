# round 6, final build: the driver's c3 command twice more on one box (run-to-run and box-to-box spread of the
# headline; the first run is profiles/r06_final/c3_bench.json)
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
for r in 2 3; do
  timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/c3_bench_rep$r.json 2> $O/c3_bench_rep$r.err || exit 1
  echo "rep $r $(python tools/r06_summary.py $O/c3_bench_rep$r.json | cut -c1-400)"
done
