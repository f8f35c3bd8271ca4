"""Floor of the A3/O3 step's data movement at a given env count (GPU box):
graph-replay time per launch of (a) an empty kernel with the block kernel's
grid, (b) a kernel that stages the step's input spans into LDS and stores
the step's output bytes with nothing in between, (c) the same with a
dependent VALU chain per lane, next to the real step kernel.

Run: python scripts/probes/floor.py [P]  (needs scripts/probes/libfloor.so:
hipcc -O3 --offload-arch=gfx950 -shared -fPIC floor_probe.hip -o libfloor.so)"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
lib = ctypes.CDLL(os.path.join(HERE, "libfloor.so"))
dev = torch.device("cuda", 0)
f = lambda n: torch.rand(n, device=dev)
u8 = lambda n: torch.zeros(n, dtype=torch.uint8, device=dev)
bufs = [f(P * 15), f(P * 6), f(P * 6), f(P * 2), f(P), u8(P),
        f(P * 36), f(P * 15), f(P), f(P), u8(P), u8(P), u8(P)]
spans = (ctypes.c_void_p * 13)(*[b.data_ptr() for b in bufs])
blocks = (P + 63) // 64


def graph_us(fn, n=25, reps=12):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / n)
    ts.sort()
    return ts[len(ts) // 2]


def launch(which, chain=0):
    def fn():
        rc = lib.floor_launch(which, blocks, spans, chain,
                              ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(0)))
        assert rc == 0, rc
    return fn


alg = 336 * P
print(f"P={P} blocks={blocks} algorithmic bytes {alg / 1e6:.2f} MB")
for name, fn in [("empty", launch(0)), ("stage+store nt", launch(1)),
                 ("stage+store plain", launch(2))] + [
        (f"stage+chain{c}+store nt", launch(1, c)) for c in (100, 300, 600, 1200)]:
    us = graph_us(fn)
    print(f"{name:28s} {us:7.2f} us/launch  {alg / us / 1e6:6.2f} TB/s", flush=True)
import marlnav_amd as pkg  # noqa: E402
env = bench.make_env(pkg, P, 3, 3, dev, 0)
acts = bench.make_actions(P, 3, dev, 0)
us, _ = bench.kernel_time_us(env, acts)
print(f"{'step kernel (block_kernel)':28s} {us:7.2f} us/launch  {alg / us / 1e6:6.2f} TB/s")
