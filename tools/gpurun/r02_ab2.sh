# A/B of a library variant on the c3 and c2 benches
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VAR=${VAR:-exp_nofwd}
for cfg in c3 c2; do
timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab_base_$cfg.log 2>&1 && \
HGX_LIB=libhgx_$VAR.so timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-ingest --no-chunked --no-check > gpurun_out/ab_${VAR}_$cfg.log 2>&1 || exit 1
done
