# k_round_pb (bases-barrier fix): pb vs steps over the probe grid, then the pb tests
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
PYTHONPATH=. timeout -k 10 400 python -u tools/probe/pb_diff.py > $O/pb1_diff.log 2>&1 || { tail -30 $O/pb1_diff.log; exit 1; }
grep -v amdgpu.ids $O/pb1_diff.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_round_pb.py -x -v --timeout 200 --timeout-method thread -k "not c5_prefix" > $O/pb1_tests.log 2>&1 || { tail -40 $O/pb1_tests.log; exit 1; }
tail -1 $O/pb1_tests.log
