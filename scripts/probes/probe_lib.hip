// The dispatch probe kernel behind a C entry point, to launch it from a
// Python/torch process (scripts/probes/probe_dispatch.py).
#include <hip/hip_runtime.h>
struct Big { float f[40]; void *p[18]; long long l[6]; };
__global__ void probe(unsigned long long *t, int nwaves_per_block, Big big)
{
    extern __shared__ float lds[];
    const unsigned long long now = wall_clock64();
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * nwaves_per_block + (threadIdx.x >> 6);
        t[2 * w] = now;
        t[2 * w + 1] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
    }
    if (big.f[0] == 12345.0f) lds[threadIdx.x] = big.f[threadIdx.x % 40];
}
extern "C" int probe_launch(void *t, int blocks, int threads, int lds, void *stream)
{
    Big big{};
    void *args[] = {&t, &threads, &big};
    int wpb = threads / 64;
    args[1] = &wpb;
    return (int)hipLaunchKernel((const void *)probe, dim3(blocks), dim3(threads), args, lds,
                                (hipStream_t)stream);
}
