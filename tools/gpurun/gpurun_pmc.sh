# one rocprofv3 PMC pass over a c3 phase_timing run: gpurun_pmc.sh <tag> <counters...>
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pmc_$tag
timeout -s KILL 150 rocprofv3 --pmc "$@" -d /tmp/pmc_$tag -o c3 -- python3 tools/phase_timing.py ${CFG:-c3} 1 > gpurun_out/pmc_$tag.log 2>&1
python3 tools/rocpd_export.py counters /tmp/pmc_$tag/c3_results.db gpurun_out/pmc_${tag}_counters.csv
