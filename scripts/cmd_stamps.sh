#!/bin/bash
# Per-phase stamps at the steady mix of finished envs, plus a same-box A/B of
# the product build against $LIBS (graph replay); every GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFGS:-65536x3x3}
WARM=${WARM:-150} B2B=${B2B:-8} timeout -k 10 120 python scripts/kstamps.py "$CFG" > gpurun_out/stamps.txt 2>&1 || exit $?
tail -n 12 gpurun_out/stamps.txt | cut -c1-1500
if [ -n "${LIBS:-}" ]; then
  timeout -k 10 300 python scripts/ab_steady.py "$CFG" marl-nav_amd/lib/libmarlnav.so $LIBS > gpurun_out/ab.txt 2>&1 || exit $?
  cat gpurun_out/ab.txt | grep -v amdgpu.ids
fi
