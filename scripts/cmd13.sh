set -u
L=marl-nav_amd/lib
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt13.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pt13.log
case $rc in 0) ;; *) exit $rc;; esac
REPS=3 timeout -k 10 300 python scripts/ab_steady.py 65536x3x3,4096x16x32,16384x3x3 $L/libmarlnav.so $L/prev.so $L/cm1.so > gpurun_out/ab13.log 2>&1; echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/ab13.log
WARM=150 B2B=8 timeout -k 10 300 python scripts/kstamps.py 65536x3x3 > gpurun_out/kstamps13.log 2>&1; echo "kstamps rc=$?"; grep -v amdgpu.ids gpurun_out/kstamps13.log | grep -E "phase_median|with_reobs|without" | cut -c1-600
