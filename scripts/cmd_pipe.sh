#!/bin/bash
# Round-6 A/B of the pipelined env-block kernel (MARLNAV_BLOCK_PIPE=2):
# GPU suite on pipe2.so (bit-exactness), then same-box graph replay of the
# working-tree product, HEAD (ref.so) and pipe2.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
MARLNAV_LIB=marl-nav_amd/lib/pipe2.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pipe2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_pipe2.log; [ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' gpurun_out/pytest_pipe2.log | head -20; exit $rc; }
fi
REPS=${REPS:-3} timeout -k 10 ${ABT:-500} python scripts/ab_steady.py ${CFGS:-65536x3x3,32768x3x3,131072x3x3,1048576x3x3} marl-nav_amd/lib/libmarlnav.so marl-nav_amd/lib/ref.so marl-nav_amd/lib/pipe2.so > gpurun_out/ab_pipe.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_pipe.txt
echo done
