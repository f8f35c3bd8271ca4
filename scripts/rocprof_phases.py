"""Split a rocprofv3 kernel trace of one bench.py run into its phases (the
step kernel's launches in order): graph-replayed prewarm, host-launched
warmup/timed/event passes, graph-replayed cross-check. Prints per phase the
launch count, mean/median duration and the median start-to-start gap.
usage: python scripts/rocprof_phases.py run_kernel_trace.csv [steps] [warmup]"""
import csv
import statistics as st
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = [r for r in csv.DictReader(open(path)) if "_kernel<" in r["Kernel_Name"]
            and ("block_kernel" in r["Kernel_Name"] or "split_kernel" in r["Kernel_Name"]
                 or "wave_kernel" in r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    s = [int(r["Start_Timestamp"]) for r in rows]
    n = len(d)
    graph_x = 3 + 12 * 8 * 25 + 25  # kernel_time_us: 3 side steps, 1 + 12*8 replays of 25
    host = warm + 2 * steps
    ph = [("prewarm (graph replays)", 0, n - graph_x - host),
          ("warmup + timed + event pass (host launches)", n - graph_x - host, n - graph_x),
          ("cross-check (graph replays)", n - graph_x, n)]
    print(f"step-kernel launches: {n}, mean {st.mean(d) / 1e3:.3f} us (rocprof's average)")
    for name, a, b in ph:
        if b - a < 2:
            continue
        x = d[a:b]
        gaps = [s[i + 1] - s[i] for i in range(a, b - 1)]
        print(f"{name}: {b - a} launches, mean {st.mean(x) / 1e3:.3f} us, median "
              f"{st.median(x) / 1e3:.3f} us, start-to-start median {st.median(gaps) / 1e3:.3f} us")


if __name__ == "__main__":
    main()
