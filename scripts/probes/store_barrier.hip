// store_barrier.hip - does a block's output store issued before a workgroup
// barrier delay the block? (DESIGN.md §5 "Where the stores go")
//
// One launch of `blocks` workgroups of 3 waves (the env-block kernel's shape).
// Waves 1-2 store 16 KiB per block (the block store's size at A3/O3), wave 0
// runs `iters` dependent FMAs (a stand-in for the per-env phase), and the
// block meets one barrier. MODE 0: no stores; 1: the stores before the
// barrier; 2: after it; 3: before it, then s_waitcnt vmcnt(0) before the
// barrier (what a hardware wait would cost). `cpol` as in the product's
// written-through stores (17 = SC0|SC1) or 0 (plain).
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

template <int MODE, int CPOL>
__global__ void __launch_bounds__(192) store_barrier_kernel(float *out, int iters, float *sink)
{
    const int tid = (int)threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    char *base = reinterpret_cast<char *>(out) + (size_t)blockIdx.x * 16384;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 16384, 0x00020000);
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i v = {tid, (int)blockIdx.x, 2, 3};
    auto stores = [&]() {
        if (w >= 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                __builtin_amdgcn_raw_buffer_store_b128(v, r, 16 * ((tid - 64) + 128 * k), 0, CPOL);
        }
    };
    if (MODE == 1 || MODE == 3) stores();
    if (MODE == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float acc = (float)tid;
    if (w == 0)
        for (int i = 0; i < iters; i += 16) {  // (16 per trip: the chain, not the loop branch)
#pragma unroll
            for (int j = 0; j < 16; ++j) acc = __builtin_fmaf(acc, 1.0001f, 0.5f);
        }
    __syncthreads();
    if (MODE == 2) stores();
    if (acc == 12345.0f) sink[0] = acc;
}

}  // namespace

extern "C" int store_barrier_launch(int mode, int cpol, float *out, int blocks, int iters,
                                    float *sink, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
#define L(M, C) hipLaunchKernelGGL((store_barrier_kernel<M, C>), dim3(blocks), dim3(192), 0, s, out, iters, sink)
    if (cpol == 17) {
        if (mode == 0) L(0, 17); else if (mode == 1) L(1, 17); else if (mode == 2) L(2, 17); else L(3, 17);
    } else {
        if (mode == 0) L(0, 0); else if (mode == 1) L(1, 0); else if (mode == 2) L(2, 0); else L(3, 0);
    }
#undef L
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
