mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-chunked > gpurun_out/b1.json 2> gpurun_out/b1.log; echo "bench rc=$?" >> gpurun_out/b1.log
HGX_LIB=libhgx_prof.so timeout -k 10 200 python -u tools/phase_timing.py c3 2 > gpurun_out/ph_c3.log 2>&1
HGX_LIB=libhgx_prof.so timeout -k 10 200 python -u tools/phase_timing.py c2 2 > gpurun_out/ph_c2.log 2>&1
tail -5 gpurun_out/b1.log
