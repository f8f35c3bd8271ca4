"""Launch the dispatch probe from a torch process; per-XCC first entry."""
import ctypes, os, sys
import numpy as np
import torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe_lib.so"))
lib.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
for blocks, threads, lds in [(820, 256, 23000), (820, 256, 0)]:
    t = torch.zeros(2 * blocks * threads // 64, dtype=torch.int64, device="cuda")
    for rep in range(10):
        t.zero_()
        torch.cuda.synchronize()
        assert lib.probe_launch(t.data_ptr(), blocks, threads, lds,
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
        torch.cuda.synchronize()
    h = t.view(-1, 2).cpu().numpy()
    e = (h[:, 0] - h[:, 0].min()) * 0.01
    x = h[:, 1] & 15
    print(blocks, threads, lds, "spread %.2f" % e.max(),
          {int(k): round(float(e[x == k].min()), 2) for k in np.unique(x)})
