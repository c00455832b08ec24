# which one-device shard rehearsals keep every workgroup resident (fallbacks = 0)
mkdir -p gpurun_out/r06
O=gpurun_out/r06/diag_w7.log
: > $O
for spec in "256 7 11" "256 7 16" "256 7 24" "256 6 10" "200 7 11" "252 7 11" "256 8 12"; do
  set -- $spec
  r=$(GPU_MAX_HW_QUEUES=$3 PYTHONPATH=tests:. timeout -k 10 120 python tests/shard_rehearsal_worker.py $1 30000 89 $2 0 0 2>&1 | tail -1 | cut -c1-400)
  echo "n=$1 W=$2 Q=$3: $r" | tee -a $O
done
