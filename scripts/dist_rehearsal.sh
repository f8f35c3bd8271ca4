#!/bin/bash
# The N>1 bench path on one GPU box: bench.py --gpus N self-launches
# torch.distributed.run; with MARLNAV_BENCH_BACKEND=gloo the ranks share the
# box's GPU and reduce on the host (2 ranks at configs[2]'s per-GPU shape, 8
# ranks at configs[4]). Rehearsal of the launcher / barrier / max-over-ranks
# path only: ranks sharing one GPU say nothing about scaling.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
MARLNAV_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/gloo2.log 2>&1 || exit $?
grep '^{' gpurun_out/gloo2.log | cut -c1-300
MARLNAV_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 8 --config 4 --steps 20 --warmup 5 > gpurun_out/gloo8.log 2>&1 || exit $?
grep '^{' gpurun_out/gloo8.log | cut -c1-300
echo done
