#!/bin/bash
# Round 3: stamps of the headline and configs[3], PMC at HEAD for both, and the
# bench line twice at the driver's shape (launch_us behind a device spin).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 65536x3x3 4096x16x32; do
  WARM=150 B2B=8 timeout -k 10 120 python scripts/kstamps.py $c > gpurun_out/stamps_r03_$c.txt 2>&1 || exit $?
  echo "stamps $c ok"
done
bash scripts/pmc_collect.sh 65536x3x3 > gpurun_out/pmc_head.log 2>&1 || exit $?
ONLY=0124 bash scripts/pmc_collect.sh 4096x16x32 > gpurun_out/pmc_c3.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bench_spin$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench_spin$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['launch_us'], r['launch_us_passes'], r['graph_replay_launch_us'])"
done
echo done
