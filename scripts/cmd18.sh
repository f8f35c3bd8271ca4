#!/bin/bash
# A/B of the per-kind re-init pass + its sub-phase stamps + the GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ab_steady.py 65536x3x3,4096x16x32,16384x3x3 marl-nav_amd/lib/libmarlnav.so marl-nav_amd/lib/prev.so > gpurun_out/ab18.log 2>&1 || exit $?
timeout -k 10 200 python scripts/diag/block_stamps.py 65536x3x3 > gpurun_out/bst18.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu18.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/ab18.log gpurun_out/bst18.log; tail -3 gpurun_out/gpu18.log
exit $rc
