// Exhaustive check, on the GPU, of two shortcuts in the pair distance and the
// normalisation that follows it (device_math.h sqrt_fast / div2_fast), over
// EVERY fp32 x in [2^-96, 2^96) (x = dx^2 + dy^2, the sqrt_fast guard range):
//   S0: sqrt_fast as shipped: y = rsq(x), s = x y, h = y / 2, e = x - s s,
//       max(s + e h, 0)                                     == sqrtf(x)
//   S1: the halving moved into the FMA's output modifier: e2 = (x - s s) / 2
//       (v_fma_f32 ... div:2), max(s + e2 y, 0)              == sqrtf(x)
//   R1: the reciprocal of den = max(sqrtf(x), 1e-12) by one Newton step from
//       y = rsq(x) instead of from v_rcp_f32(den)            == 1 / den
//   R2: the same with two Newton steps from y                == 1 / den
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 sqrt_rcp_exhaustive.hip -o sqrt_rcp_exhaustive
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float fma_half(float a, float b, float c)
{
    float r;
    asm volatile("v_fma_f32 %0, %1, %2, %3 div:2" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__global__ void run(uint32_t lo, uint32_t n, unsigned long long *cnt, uint32_t *ex)
{
    unsigned long long b0 = 0, b1 = 0, b2 = 0, b3 = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float x = __uint_as_float(lo + i);
        const float ref = __builtin_sqrtf(x);
        const float y = __builtin_amdgcn_rsqf(x);
        const float s = x * y, h = 0.5f * y;
        const float e = __builtin_fmaf(-s, s, x);
        const float s0 = __builtin_fmaxf(__builtin_fmaf(e, h, s), 0.0f);
        const float e2 = fma_half(-s, s, x);
        const float s1 = __builtin_fmaxf(__builtin_fmaf(e2, y, s), 0.0f);
        const float den = __builtin_fmaxf(ref, 1e-12f);
        const float r1 = __builtin_fmaf(__builtin_fmaf(-den, y, 1.0f), y, y);
        const float r2 = __builtin_fmaf(__builtin_fmaf(-den, r1, 1.0f), r1, r1);
        const bool f0 = __float_as_uint(s0) != __float_as_uint(ref);
        const bool f1 = __float_as_uint(s1) != __float_as_uint(ref);
        const bool f2 = __float_as_uint(r1) != __float_as_uint(1.0f / den);
        b0 += f0;
        b1 += f1;
        b2 += f2;
        b3 += __float_as_uint(r2) != __float_as_uint(1.0f / den);
        if ((f1 || f2) && *(volatile unsigned long long *)&cnt[3] < 16) {
            const unsigned long long k = atomicAdd(&cnt[3], 1ull);
            if (k < 16) { ex[3 * k] = lo + i; ex[3 * k + 1] = __float_as_uint(f1 ? s1 : r1); ex[3 * k + 2] = f1 ? 1 : 2; }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        b0 += __shfl_xor(b0, o);
        b1 += __shfl_xor(b1, o);
        b2 += __shfl_xor(b2, o);
        b3 += __shfl_xor(b3, o);
    }
    if ((threadIdx.x & 63) == 0) {
        if (b0) atomicAdd(&cnt[0], b0);
        if (b1) atomicAdd(&cnt[1], b1);
        if (b2) atomicAdd(&cnt[2], b2);
        if (b3) atomicAdd(&cnt[4], b3);
    }
}

int main()
{
    const uint32_t lo = (uint32_t)(127 - 96) << 23, hi = (uint32_t)(127 + 96) << 23;
    unsigned long long *cnt;
    uint32_t *ex;
    hipMalloc(&cnt, 5 * sizeof(unsigned long long));
    hipMalloc(&ex, 48 * sizeof(uint32_t));
    hipMemset(cnt, 0, 5 * sizeof(unsigned long long));
    hipLaunchKernelGGL(run, dim3(8192), dim3(256), 0, 0, lo, hi - lo, cnt, ex);
    if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "launch failed\n"); return 1; }
    unsigned long long h[5];
    uint32_t e[48];
    hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost);
    hipMemcpy(e, ex, sizeof e, hipMemcpyDeviceToHost);
    printf("x in [2^-96, 2^96): %u values; S0 (shipped sqrt_fast) fails %llu, S1 (div:2 FMA) fails %llu, "
           "R1 (rsq-started reciprocal) fails %llu, R2 (two Newton steps) fails %llu\n", hi - lo, h[0], h[1],
           h[2], h[4]);
    for (unsigned long long k = 0; k < (h[3] < 16 ? h[3] : 16); ++k)
        printf("example %s x=0x%08x got=0x%08x\n", e[3 * k + 2] == 1 ? "S1" : "R1", e[3 * k], e[3 * k + 1]);
    return 0;
}
