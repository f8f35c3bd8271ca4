"""Floor references for the step kernel's timing method: per-launch HIP-event
time of (a) an empty-ish elementwise kernel and (b) device copies moving the
same bytes as one step (read 121 B + write 215 B per env at A3/O3), via
hipGraph replay of back-to-back launches and per-launch events."""
import sys, torch
P = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rd, wr = 121 * P, 215 * P
src = torch.empty(rd // 4, device="cuda")
dst = torch.empty(wr // 4, device="cuda")
tiny = torch.empty(64, device="cuda")
def graph_time(fn, n=25, reps=12):
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3): fn()
    torch.cuda.current_stream().wait_stream(s); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n): fn()
    g.replay(); torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record(); g.replay(); b.record(); b.synchronize(); ts.append(a.elapsed_time(b) * 1e3 / n)
    ts.sort(); return ts[len(ts) // 2]
def copy_rw():
    # read rd bytes, write wr bytes: write = broadcast-ish fill from the read
    dst[: rd // 4].copy_(src)
    dst[rd // 4:].fill_(1.0)
print(f"P={P} read={rd/1e6:.2f}MB write={wr/1e6:.2f}MB")
print("fill tiny     graph us/launch %.2f" % graph_time(lambda: tiny.fill_(1.0)))
print("copy rd->dst  graph us/launch %.2f" % graph_time(lambda: dst[: rd // 4].copy_(src)))
print("fill wr       graph us/launch %.2f" % graph_time(lambda: dst.fill_(1.0)))
print("copy+fill     graph us/step   %.2f" % graph_time(copy_rw))
big = torch.empty((rd + wr) // 8, device="cuda"); big2 = torch.empty((rd + wr) // 8, device="cuda")
print("copy (rd+wr)/2 each way graph us %.2f" % graph_time(lambda: big2.copy_(big)))
