# final state: full GPU suite, default bench line (c3, all legs), every other config, rocprofv3 trace + PMC of c3
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && \
for cfg in c1 c2 c4 c5; do timeout -k 10 400 python -u bench.py --config $cfg > gpurun_out/cfg_$cfg.log 2>&1 || exit 1; done && \
HGX_LIB=libhgx_prof.so timeout -k 10 200 python -u tools/phase_timing.py c3 1 > gpurun_out/prof_phases.log 2>&1 && \
bash tools/gpurun/r02_profile.sh
