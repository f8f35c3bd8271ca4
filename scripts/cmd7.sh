set -u
L=marl-nav_amd/lib
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt7.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pt7.log
REPS=3 timeout -k 10 300 python scripts/ab_steady.py 65536x3x3 $L/libmarlnav.so $L/ab2.so $L/ab4096.so $L/ab8192.so $L/ab16.so $L/cm1.so > gpurun_out/ab6.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab6.log | grep -v amdgpu.ids
LIBS="$L/libmarlnav.so $L/ra1c5403.so $L/r4ec1018.so $L/rfd06335.so $L/r7078fd9.so $L/rcf41be2.so" ONLY=014 timeout -k 10 600 bash scripts/pmc_ab.sh 4096x16x32 2>&1 | grep -v "pass"
