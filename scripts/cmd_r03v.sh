#!/bin/bash
# Round 3: GPU tests, split-kernel tail A/B against ref.so, the headline's
# stage ablations (AB 256 no draws, 128 no sin/cos, 384 neither), stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_v.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_v.log; [ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' gpurun_out/pytest_v.log | head -20; exit $rc; }
L=marl-nav_amd/lib
REPS=3 timeout -k 10 400 python scripts/ab_steady.py 4096x16x32,512x16x32 $L/libmarlnav.so $L/ref.so > gpurun_out/ab_v1.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_v1.txt
REPS=3 timeout -k 10 400 python scripts/ab_steady.py 65536x3x3,16384x3x3 $L/libmarlnav.so $L/ab256.so $L/ab128.so $L/ab384.so > gpurun_out/ab_v2.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_v2.txt
WARM=150 B2B=8 WPB=4 timeout -k 10 120 python scripts/kstamps.py 4096x16x32 > gpurun_out/stamps_v.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stamps_v.txt | tail -8 | cut -c1-700
echo done
