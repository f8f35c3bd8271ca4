#!/bin/bash
# GPU tests (optional), then a same-box A/B (graph replay, steady mix of
# finished envs) of the product build against $LIBS at $CFGS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu.txt 2>&1
  rc=$?; tail -n 8 gpurun_out/pytest_gpu.txt | cut -c1-400; [ $rc = 0 ] || exit $rc
fi
L=marl-nav_amd/lib
args=""; for x in ${LIBS:-}; do args="$args $L/$x"; done
timeout -k 10 500 python scripts/ab_steady.py "${CFGS:-65536x3x3}" $L/libmarlnav.so $args > gpurun_out/ab.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab.txt; exit $rc
