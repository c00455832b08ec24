# round 6, final build: evidence for c4 and c5, then the chunked schedule's per-call profile at c3 -> gpurun_out/r06f/
CFGS="c4 c5" bash tools/gpurun/r06_final.sh && bash tools/gpurun/r06_chunkprof.sh
