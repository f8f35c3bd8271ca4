#!/bin/bash
# Exploration session (round 4): optional stamps at $STAMPS configs, family
# A/B at $FAM shapes, steady A/B of the product build against $LIBS at $CFGS.
# Every GPU step has its own time limit; a fault / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${TAG:-x}
run() {  # name limit cmd...
    local name=$1 lim=$2; shift 2
    timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_$name.txt" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; grep -v amdgpu.ids "$OUT/${TAG}_$name.txt" | tail -n ${TAILN:-40} | cut -c1-${CUT:-700}
    [ $rc = 0 ] || exit $rc
}
[ -n "${TESTS:-}" ] && run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"}
[ -n "${STAMPS:-}" ] && WARM=${WARM:-150} B2B=${B2B:-8} run stamps 200 python scripts/kstamps.py "$STAMPS"
[ -n "${FAM:-}" ] && run family 300 python scripts/diag/family_ab.py $FAM
if [ -n "${LIBS:-}" ]; then
  args=""; for x in $LIBS; do args="$args marl-nav_amd/lib/$x"; done
  run ab 600 python scripts/ab_steady.py "${CFGS:-65536x3x3}" marl-nav_amd/lib/libmarlnav.so $args
fi
echo done
