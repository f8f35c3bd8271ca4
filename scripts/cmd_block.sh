export TMPDIR=/tmp
L=marl-nav_amd/lib
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pt.log
timeout -k 10 200 python scripts/graph_time.py ${CFGS:-65536x3x3,16384x3x3,2097152x3x3,65536x3x8} $L/blk_e0_s1.so $L/blk_rr.so $L/libmarlnav.so > gpurun_out/gt1.log 2>&1 || exit 1
[ "${STAMPS:-1}" = 1 ] && B2B=8 timeout -k 10 120 python scripts/kstamps.py 65536x3x3,16384x3x3 > gpurun_out/kst_blk.log 2>&1
exit 0
