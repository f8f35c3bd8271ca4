"""Summarise scripts/valu_census.sh: counters per wave of the step kernel for
each build, and the per-phase differences between consecutive truncation
builds (given in kernel order). usage: census_summarize.py DIR tag:lib ..."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summarize_lib import is_step  # noqa: E402

out, specs = sys.argv[1], sys.argv[2:]
tags = [s.split(":", 1)[0] for s in specs]
per_wave = {}
for tag in tags:
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(out, tag, "p*", "run_counter_collection.csv"))):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if not is_step(r["Kernel_Name"]):
                continue
            d = per[r["Counter_Name"]]
            d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        waves = per.pop("SQ_WAVES", None)
        for k, v in per.items():
            ids = sorted(v)[5:]  # skip warm-up dispatches
            if ids and waves:
                acc[k].append(sum(v[i] / waves[i] for i in ids) / len(ids))
    per_wave[tag] = {k: sum(v) / len(v) for k, v in acc.items()}
keys = sorted({k for t in per_wave.values() for k in t})
short = lambda k: k.replace("SQ_INSTS_", "").replace("SQ_", "")
print("per wave".ljust(14) + "".join(f"{short(k):>13s}" for k in keys))
for t in tags:
    print(t.ljust(14) + "".join(f"{per_wave[t].get(k, float('nan')):13.1f}" for k in keys))
print("differences (phase = later build - earlier build)")
for a, b in zip(tags, tags[1:]):
    print(f"{b}-{a}"[:14].ljust(14) + "".join(
        f"{per_wave[b].get(k, 0) - per_wave[a].get(k, 0):13.1f}" for k in keys))
json.dump(per_wave, open(os.path.join(out, "census.json"), "w"), indent=1, sort_keys=True)
