# the full GPU suite, the default bench line, the chunked-call probe, then the rocprofv3 kernel trace and PMC traffic
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u tools/probe/chunk_calls.py 256 1000000 1000 > gpurun_out/chunk_calls.log 2>&1 && \
HGX_LIB=libhgx_prof.so timeout -k 10 200 python -u tools/phase_timing.py c3 1 > gpurun_out/prof_phases.log 2>&1 && \
bash tools/gpurun/r02_profile.sh
