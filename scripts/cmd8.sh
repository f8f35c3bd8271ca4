set -u
L=marl-nav_amd/lib
REPS=3 timeout -k 10 300 python scripts/ab_steady.py 65536x3x3 $L/libmarlnav.so $L/ab32768.so $L/ab65536.so $L/ab131072.so $L/ab4096.so > gpurun_out/ab8.log 2>&1; echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/ab8.log
REPS=3 timeout -k 10 300 python scripts/ab_steady.py 4096x16x32,512x16x32,1024x3x8 $L/libmarlnav.so $L/nopad.so > gpurun_out/ab8b.log 2>&1; echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/ab8b.log
LIBS="$L/libmarlnav.so $L/nopad.so" ONLY=014 timeout -k 10 300 bash scripts/pmc_ab.sh 4096x16x32 2>&1 | grep -v "pass"
