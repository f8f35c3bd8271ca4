# parity suite, then graph-replay A/B of libmarlnav.so against other builds
# (scripts/build_variant.sh makes them; LIBS lists them, CFGS the configs)
export TMPDIR=/tmp
L=marl-nav_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python scripts/graph_time.py ${CFGS:-4096x16x32,512x16x32,1024x3x8,65536x3x3} $L/libmarlnav.so ${LIBS:-$L/ref.so} > gpurun_out/ab.log 2>&1
