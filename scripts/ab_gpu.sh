#!/bin/bash
# GPU tests of the working tree (TESTS=0: none), then a same-box A/B of
# libmarlnav.so against $LIBS at $CFGS (graph replay, steady mix):
#   CFGS=65536x3x3,4096x16x32 LIBS=marl-nav_amd/lib/ref.so bash scripts/ab_gpu.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_w.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_w.log; [ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' gpurun_out/pytest_w.log | head -20; exit $rc; }
fi
libs=""; for x in ${LIBS:-}; do case $x in */*) libs="$libs $x";; *) libs="$libs marl-nav_amd/lib/$x";; esac; done
REPS=${REPS:-3} timeout -k 10 ${ABT:-500} python scripts/ab_steady.py $CFGS marl-nav_amd/lib/libmarlnav.so $libs > gpurun_out/ab_w.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_w.txt
echo done
