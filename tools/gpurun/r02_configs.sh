# the default bench line of every config (c1 c2 c4 c5; c3 is the default run)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in c1 c2 c4 c5; do
  timeout -k 10 400 python -u bench.py --config $cfg > gpurun_out/cfg_$cfg.log 2>&1 || exit 1
done
