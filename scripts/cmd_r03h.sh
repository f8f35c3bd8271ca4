TAG=r03h bash scripts/gpu_r03.sh && \
timeout -k 10 300 python scripts/graph_time.py 2x3x3,1024x3x8,65536x3x3,4096x16x32,16384x3x3,131072x3x8 > gpurun_out/configs_r03h.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4_r03h -o run -- python scripts/pmc_run.py 4096x16x32 40 > gpurun_out/prof_c4_r03h.log 2>&1; echo rc=$?
