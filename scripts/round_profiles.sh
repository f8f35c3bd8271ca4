#!/bin/bash
# Round-end measurement set (one GPU box): parity tests, smoke, the bench line
# with its CPU baseline, rocprofv3 kernel stats of the bench, PMC counters of
# the headline config, graph-replay step times of every BASELINE config, and a
# kernel-stats profile of a large-P (HBM-bound) run. Outputs under
# gpurun_out/; copy the summaries into profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out
mkdir -p $OUT
TAG=$TAG PROFILE=1 bash scripts/gpu_check.sh || exit $?
bash scripts/pmc_collect.sh 65536x3x3 || exit $?
timeout -k 10 300 python scripts/graph_time.py 2x3x3,1024x3x8,65536x3x3,4096x16x32,16384x3x3,2097152x3x3 \
    > $OUT/configs_$TAG.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_large_$TAG -o run \
    -- python scripts/pmc_run.py 2097152x3x3 40 > $OUT/prof_large_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4_$TAG -o run \
    -- python scripts/pmc_run.py 4096x16x32 40 > $OUT/prof_c4_$TAG.log 2>&1 || exit $?
echo round_profiles done
