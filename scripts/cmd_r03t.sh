#!/bin/bash
# Round 3: per-wave stamps of the finished-env tail, and the tail's ablations
# (AB 1: no re-init, AB 16: re-init without pair math) in a same-box A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WARM=150 B2B=8 WPB=3 timeout -k 10 120 python scripts/kstamps.py 65536x3x3 > gpurun_out/stamps_r03b_65536x3x3.txt 2>&1 || exit $?
WARM=150 B2B=8 WPB=4 timeout -k 10 120 python scripts/kstamps.py 4096x16x32 > gpurun_out/stamps_r03b_4096x16x32.txt 2>&1 || exit $?
grep 'with_reobs wave' gpurun_out/stamps_r03b_*.txt | cut -c1-600
REPS=3 timeout -k 10 400 python scripts/ab_steady.py 65536x3x3,4096x16x32,16384x3x3 marl-nav_amd/lib/libmarlnav.so marl-nav_amd/lib/ab1.so marl-nav_amd/lib/ab16.so > gpurun_out/ab_tail.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_tail.txt
echo done
