#!/bin/bash
# Round-3 end evidence (one GPU box): GPU tests, smoke, the bench line at the
# driver's shape (twice) and at 500 steps with the CPU baseline, rocprofv3
# kernel stats of the bench and of configs[3], PMC of both, graph-replay step
# times of every BASELINE config. Each GPU step has its own time limit; a
# fault / abort / timeout ends the script. Copy the outputs into profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r03_final}
mkdir -p "$OUT"
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() {  # name timeout cmd...
    local name=$1 lim=$2; shift 2
    timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    grep -v amdgpu.ids "$OUT/${TAG}_$name.log" | tail -${TAILN:-3} | cut -c1-400
    if fatal $rc; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    [ $rc -eq 0 ] || { echo "failed: $name"; exit 1; }
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_drv1 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off
step bench_drv2 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off
step bench_500 300 python bench.py --steps 500 --warmup 50
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python bench.py --steps 200 --warmup 20 --cpu-baseline off
step rocprof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3_$TAG -o run \
    -- python scripts/pmc_run.py 4096x16x32 200
step graph 300 python scripts/graph_time.py 2x3x3,1024x3x8,65536x3x3,4096x16x32,16384x3x3,131072x3x8,2097152x3x3
bash scripts/pmc_collect.sh 65536x3x3 > $OUT/${TAG}_pmc_head.log 2>&1 || exit $?
bash scripts/pmc_collect.sh 4096x16x32 > $OUT/${TAG}_pmc_c3.log 2>&1 || exit $?
echo round_end done
