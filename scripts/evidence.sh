#!/bin/bash
# A round's evidence set on one GPU box (TAG names it, e.g. TAG=r06_end):
# GPU tests, smoke, the bench line at the
# driver's shape (twice) and at 500 steps with the CPU baseline, rocprofv3
# kernel stats of the bench at configs[2] and at configs[4]'s per-GPU shape
# and of configs[3], graph-replay step times of every BASELINE config, PMC of
# configs[2] / configs[4] per GPU / configs[3], and the N>1 bench path
# rehearsed over gloo with ranks sharing the one GPU. Every GPU step has its
# own time limit; a fault / abort / timeout ends the script. Switches:
# TESTS SMOKE BENCH PROF GRAPH PMC DIST (1 = run, default 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-evidence}
mkdir -p "$OUT"
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() {  # name timeout cmd...
    local name=$1 lim=$2; shift 2
    echo "== $name"
    timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    grep -v amdgpu.ids "$OUT/${TAG}_$name.log" | tail -${TAILN:-4} | cut -c1-${CUT:-600}
    if fatal $rc; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    [ $rc -eq 0 ] || { echo "failed: $name"; exit 1; }
}
on() { [ "${!1:-1}" = 1 ]; }
on TESTS && step pytest_gpu 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
on SMOKE && step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
if on BENCH; then
  step bench_drv1 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off
  step bench_drv2 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off
  step bench_500 300 python bench.py --steps 500 --warmup 50
fi
if on PROF; then
  step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
      -- python bench.py --steps 200 --warmup 20 --cpu-baseline off
  step rocprof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4_$TAG -o run \
      -- python bench.py --envs 16384 --steps 200 --warmup 20 --cpu-baseline off
  step rocprof_2m 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_2m_$TAG -o run \
      -- python scripts/pmc_run.py 2097152x3x3 300
  step rocprof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3_$TAG -o run \
      -- python scripts/pmc_run.py 4096x16x32 200
fi
on GRAPH && step graph 300 python scripts/graph_time.py 2x3x3,1024x3x8,65536x3x3,4096x16x32,16384x3x3,32768x3x3,131072x3x8,2097152x3x3
if on PMC; then
  for c in 65536x3x3 16384x3x3 4096x16x32; do
    bash scripts/pmc_collect.sh $c > $OUT/${TAG}_pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
    echo "== pmc $c"; tail -3 $OUT/${TAG}_pmc_$c.log
  done
fi
if on DIST; then
  MARLNAV_BENCH_BACKEND=gloo step bench_gloo2 300 python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-seconds 3
  step bench_gloo8_c4 400 python bench.py --gpus 8 --config 4 --steps 20 --warmup 5 --cpu-seconds 3
fi
echo evidence done
