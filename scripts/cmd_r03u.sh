#!/bin/bash
# Round 3: GPU tests of the working tree, then a same-box A/B against $REF
# (graph replay, steady mix) and the per-wave stamps of configs[3].
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_u.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_u.log; [ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' gpurun_out/pytest_u.log | head -20; exit $rc; }
REPS=${REPS:-3} timeout -k 10 400 python scripts/ab_steady.py ${CFGS:-4096x16x32,512x16x32,65536x3x3} marl-nav_amd/lib/libmarlnav.so ${REF:-marl-nav_amd/lib/ref.so} > gpurun_out/ab_u.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_u.txt
if [ "${STAMPS:-1}" = 1 ]; then
WARM=150 B2B=8 WPB=4 timeout -k 10 120 python scripts/kstamps.py 4096x16x32 > gpurun_out/stamps_u.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stamps_u.txt | tail -8 | cut -c1-700
fi
echo done
