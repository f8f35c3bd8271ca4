set -u
L=marl-nav_amd/lib
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt10.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt10.log
case $rc in 0|1) ;; *) exit $rc;; esac
INPLACE=inplace.so REPS=3 timeout -k 10 300 python scripts/ab_steady.py 65536x3x3,4096x16x32,16384x3x3,1024x3x8,2x3x3 $L/libmarlnav.so $L/inplace.so $L/cm1.so > gpurun_out/ab10.log 2>&1; echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/ab10.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/b10_20.log 2>&1; tail -1 gpurun_out/b10_20.log | cut -c1-300
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03_pp -o run -- python bench.py --steps 200 --warmup 20 --cpu-baseline off > gpurun_out/prof10.log 2>&1; echo "prof rc=$?"; head -2 gpurun_out/prof_r03_pp/run_kernel_stats.csv | cut -c1-250
