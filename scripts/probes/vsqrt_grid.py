"""v_sqrt_f32 on the r-grid of the library acosf (k * 2^-25, k < 2^23) against
the correctly rounded sqrt (GPU box). Writes gpurun_out/vsqrt_grid.npy (the
raw fp32 results) and gpurun_out/vsqrt_r_grid.npz, the generating run of the
fixture tests/golden/vsqrt_r_grid.npz: `down` = bit k (little-endian packed)
set where v_sqrt_f32(k * 2^-25) is one ulp below the correctly rounded sqrt,
`up` = the k where it is one ulp above (the oracle's acos_device applies
them: oracle/marlnav_oracle.c). Prints the error structure."""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "probes", "libacos.so"))
lib.vsqrt_grid.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
N = 1 << 23
buf = torch.empty(N, dtype=torch.float32, device="cuda")
assert lib.vsqrt_grid(0, N, buf.data_ptr(), None) == 0
v = buf.cpu().numpy()
k = np.arange(N, dtype=np.float64)
r = (k * 2.0 ** -25).astype(np.float32)
assert np.array_equal(r.astype(np.float64), k * 2.0 ** -25)
cr = np.sqrt(r.astype(np.float64)).astype(np.float32)
d = v.view(np.int32).astype(np.int64) - cr.view(np.int32).astype(np.int64)
print("ulp differences:", dict(zip(*[x.tolist() for x in np.unique(d, return_counts=True)])))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", "vsqrt_grid.npy"), v)
bad = np.flatnonzero(d)
print("first mismatching k:", bad[:10].tolist(), "last:", bad[-5:].tolist())
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "vsqrt_r_grid.npz"),
                    down=np.packbits(d == -1, bitorder="little"),
                    up=np.flatnonzero(d == 1).astype(np.uint32), n=np.int64(N))
assert set(np.unique(d).tolist()) <= {-1, 0, 1}, "v_sqrt_f32 more than one ulp off"
