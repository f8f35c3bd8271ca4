set -u
L=marl-nav_amd/lib
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt17.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pt17.log
case $rc in 0) ;; *) exit $rc;; esac
REPS=3 timeout -k 10 300 python scripts/ab_steady.py 65536x3x3,4096x16x32,16384x3x3,1024x3x8 $L/libmarlnav.so $L/norefc.so $L/cm1.so $L/prev.so > gpurun_out/ab17.log 2>&1; echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/ab17.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/b17.log 2>&1; tail -1 gpurun_out/b17.log | cut -c1-200
WARM=150 B2B=8 timeout -k 10 300 python scripts/kstamps.py 65536x3x3 > gpurun_out/kstamps17.log 2>&1; echo "kstamps rc=$?"; grep -v amdgpu.ids gpurun_out/kstamps17.log | grep -E "phase_median|with_reobs|without" | cut -c1-600
