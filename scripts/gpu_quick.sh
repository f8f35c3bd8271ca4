#!/bin/bash
# Quick GPU iteration: parity tests (optionally a -k filter), smoke, short benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() {
    local name=$1 lim=$2; shift 2
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-4} | cut -c1-${CUT:-600}
    if fatal $rc; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
[ "${TESTS:-1}" = 1 ] && step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"}
[ "${SMOKE:-1}" = 1 ] && step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
[ "${BENCH:-1}" = 1 ] && {
  step bench_drv1 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off
  step bench_drv2 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off
  step bench_500 200 python bench.py --steps 500 --warmup 50 ${CPUB:---cpu-baseline off}
}
[ "${GLOO2:-0}" = 1 ] && MARLNAV_BENCH_BACKEND=gloo step bench_gloo2 300 python bench.py --gpus 2 --steps 20 --warmup 5
exit 0
