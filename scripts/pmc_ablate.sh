#!/bin/bash
# Instruction counts per wave (one PMC pass) of the step kernel for each
# library given (ablation builds), at one config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-65536x3x3}
for lib in "$@"; do
  tag=$(basename $lib .so)
  OUT=gpurun_out/pmca_$tag
  rm -rf $OUT; mkdir -p $OUT
  MARLNAV_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES --output-format csv -d $OUT/p0 -o run -- python scripts/pmc_run.py $CFG 40 > $OUT/p0.log 2>&1
  rc=$?
  case $rc in 0|1) ;; *) echo "$tag rc=$rc"; exit $rc;; esac
  python - $OUT $tag <<'PY'
import csv, glob, sys, collections
out, tag = sys.argv[1], sys.argv[2]
per = collections.defaultdict(dict)
for f in glob.glob(out + "/p0/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if ("wave_kernel" not in n and "tile_kernel" not in n) or "true" in n.split(",")[2]:
            continue
        per[r["Counter_Name"]][r["Dispatch_Id"]] = per[r["Counter_Name"]].get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
avg = {k: sum(list(v.values())[5:]) / max(1, len(v) - 5) for k, v in per.items()}
w = avg.get("SQ_WAVES", 1)
print(tag, " ".join(f"{k[8:] if k.startswith('SQ_INSTS') else k}={avg[k]/w:.1f}" for k in sorted(avg) if k != "SQ_WAVES"), f"waves={w:.0f}")
PY
done
