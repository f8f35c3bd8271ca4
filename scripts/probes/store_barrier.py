"""GPU box: hipGraph-replay time of store_barrier.hip's kernel per mode
(0 no stores, 1 before the barrier, 2 after it, 3 before it + vmcnt(0)), at
1024 and 256 blocks (65536 / 16384 envs' block counts), written-through and
plain stores, two lengths of wave 0's dependent FMA chain."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libstore_barrier.so"))
lib.store_barrier_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]


def replay_us(mode, cpol, blocks, iters, out, sink, n=25, reps=8):
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for _ in range(3):
            assert lib.store_barrier_launch(mode, cpol, out.data_ptr(), blocks, iters, sink.data_ptr(),
                                            ctypes.c_void_p(s.cuda_stream)) == 0
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            lib.store_barrier_launch(mode, cpol, out.data_ptr(), blocks, iters, sink.data_ptr(),
                                     ctypes.c_void_p(s.cuda_stream))
    g.replay()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(4):
            g.replay()
        b.record()
        b.synchronize()
        t.append(a.elapsed_time(b) * 1e3 / (4 * n))
    t.sort()
    return t[len(t) // 2]


def main():
    out = torch.zeros(1024 * 4096, dtype=torch.float32, device="cuda")
    sink = torch.zeros(1, dtype=torch.float32, device="cuda")
    for blocks in (1024, 256):
        for iters in (200, 800):
            for cpol in (17, 0):
                row = [replay_us(m, cpol, blocks, iters, out, sink) for m in (0, 1, 2, 3)]
                print(f"blocks {blocks:5d} fma {iters:4d} cpol {cpol:2d}  none {row[0]:.2f}  "
                      f"before {row[1]:.2f}  after {row[2]:.2f}  before+vmcnt0 {row[3]:.2f} us",
                      flush=True)


if __name__ == "__main__":
    main()
