#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r02}
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

step() {  # name timeout cmd...
    local name=$1 lim=$2; shift 2
    echo "== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -5 "$OUT/$name.log"
    if fatal $rc; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}

rocminfo 2>/dev/null | grep -m2 -E "Marketing Name|gfx" > "$OUT/device.txt" || true
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 500 --warmup 50
step bench_drv 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off
if [ "${PROFILE:-1}" = 1 ]; then
  step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_$TAG" -o run -- python bench.py --steps 200 --warmup 20 --cpu-baseline off
fi
echo done
