#!/bin/bash
# Round-3 GPU session: parity tests, smoke, driver-shaped and long benches,
# the N>1 bench path rehearsed with gloo on the one GPU (2 ranks; configs[4]
# as 8 ranks), and rocprofv3 kernel stats. Each GPU step has its own limit;
# a fault / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r03}
mkdir -p "$OUT"
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() {  # name timeout cmd...
    local name=$1 lim=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    grep -v amdgpu.ids "$OUT/${TAG}_$name.log" | tail -${TAILN:-6} | cut -c1-${CUT:-2000}
    if fatal $rc; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
[ "${TESTS:-1}" = 1 ] && step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"}
[ "${SMOKE:-1}" = 1 ] && step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
if [ "${BENCH:-1}" = 1 ]; then
  step bench_drv1 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off
  step bench_drv2 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off
  step bench_500 300 python bench.py --steps 500 --warmup 50 ${CPUB:-}
fi
if [ "${DIST:-0}" = 1 ]; then
  MARLNAV_BENCH_BACKEND=gloo step bench_gloo2 300 python bench.py --gpus 2 --steps 20 --warmup 5
  MARLNAV_BENCH_BACKEND=gloo step bench_gloo8_c4 300 python bench.py --gpus 8 --config 4 --steps 20 --warmup 5
fi
if [ "${PROF:-1}" = 1 ]; then
  step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_${TAG}" -o run -- python bench.py --steps 200 --warmup 20 --cpu-baseline off
  head -3 "$OUT/prof_${TAG}/run_kernel_stats.csv" | cut -c1-250
fi
echo done
