# round 6: the whole GPU suite on the default build (one process), then smoke()
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite_${TAG:-a}.log 2>&1 \
  || { tail -60 $O/suite_${TAG:-a}.log; exit 1; }
tail -3 $O/suite_${TAG:-a}.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_${TAG:-a}.log 2>&1 || { tail -20 $O/smoke_${TAG:-a}.log; exit 1; }
tail -2 $O/smoke_${TAG:-a}.log
