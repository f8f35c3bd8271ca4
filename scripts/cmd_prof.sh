#!/bin/bash
# bench line + rocprofv3 kernel stats of the same bench command (graph-replayed
# prewarm), per-phase split of the trace; every GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03p}
mkdir -p gpurun_out
ARGS=${ARGS:---steps 20 --warmup 5 --cpu-baseline off}
timeout -k 10 200 python bench.py $ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
cat gpurun_out/${TAG}_bench.json | cut -c1-1500
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python bench.py $ARGS > gpurun_out/${TAG}_rocprof.log 2>&1 || exit $?
head -3 gpurun_out/prof_${TAG}/run_kernel_stats.csv | cut -c1-300
python scripts/rocprof_phases.py gpurun_out/prof_${TAG}/run_kernel_trace.csv
