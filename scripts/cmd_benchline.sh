#!/bin/bash
# The bench line at the driver's shape (twice, with the CPU baseline), at 500
# steps, and a rocprofv3 kernel-stats run of the 20-step command; prints
# value, ms_per_step, roofline.launch_us / frac / timed_region_frac and the
# rocprof average of the step kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bf$i.log 2>&1 || exit 1; done
timeout -k 10 200 python bench.py --steps 500 --warmup 50 --cpu-baseline off > gpurun_out/bf3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bf -o run \
    -- python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bf4.log 2>&1 || exit 1
python3 - <<'PY'
import csv, json
for f in ["gpurun_out/bf1.log", "gpurun_out/bf2.log", "gpurun_out/bf3.log", "gpurun_out/bf4.log"]:
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            r = d["roofline"]
            cpu = d["cpu_baseline"]
            print(f, d["steps"], round(d["value"] / 1e9, 3), round(d["ms_per_step"] * 1e3, 3),
                  "launch_us", round(r["launch_us"], 3), "frac", round(r["frac"], 3),
                  "timed", round(r["timed_region_frac"], 3), "cpu", None if cpu is None else round(cpu["value"]))
for r in csv.DictReader(open("gpurun_out/prof_bf/run_kernel_stats.csv")):
    if "block_kernel" in r["Name"]:
        print("rocprof", r["Calls"], r["AverageNs"])
PY
