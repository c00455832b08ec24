# round 6, final build: evidence for c3, c1, c2 (PMC traffic + VALU, rocprofv3 kernel stats, the bench line of the
# driver's command for c3) -> gpurun_out/r06f/
CFGS="c3 c1 c2" bash tools/gpurun/r06_final.sh
