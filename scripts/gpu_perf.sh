#!/bin/bash
# GPU perf iteration: parity tests, probes, stamps, kbench, rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-perf}
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() {
    local name=$1 lim=$2; shift 2
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-12}
    if fatal $rc; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
L=marl-nav_amd/lib
[ "${TESTS:-1}" = 1 ] && TAILN=3 step pytest_gpu 600 python -m pytest tests -m gpu -x -q
[ -x scripts/probes/div_probe ] && [ "${DIVPROBE:-0}" = 1 ] && step div_probe 300 scripts/probes/div_probe
[ "${STAMPS:-1}" = 1 ] && step kstamps 200 python scripts/kstamps.py ${CONFIGS:-65536x3x3,2097152x3x3}
step kbench 300 python scripts/kbench.py --configs ${CONFIGS:-65536x3x3,2097152x3x3,4096x16x32,1024x3x8} --lib $L/libmarlnav.so ${EXTRA_LIBS:-}
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python scripts/kbench.py --configs ${CONFIGS:-65536x3x3,2097152x3x3,4096x16x32,1024x3x8} --rounds 1 --launches 50
python - <<'PY'
import csv, glob, collections
rows = list(csv.DictReader(open(glob.glob("gpurun_out/prof_*/run_kernel_trace.csv")[-1])))
by = collections.defaultdict(list)
for r in rows:
    if any(k in r["Kernel_Name"] for k in ("wave_kernel", "tile_kernel", "split_kernel")):
        by[(r["Kernel_Name"][:60], r.get("Grid_Size", r.get("Grid_Size_X")))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in by.items():
    v.sort()
    print("rocprof", k[1], "grid", "n=%d median_us=%.2f min=%.2f" % (len(v), v[len(v)//2], v[0]), k[0])
PY
