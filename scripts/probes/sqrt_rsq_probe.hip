// Exhaustive check of shorter correctly rounded sqrt candidates over every
// float of sqrt_fast's range [2^-96, 2^96] and zero (the FAST pair math):
//   A: y = v_rsq(x); s = x*y; h = 0.5*y; e = fma(-s, s, x); r = fma(e, h, s); max(r, 0)
//   B: s = v_sqrt(x); y = v_rsq(x); e = fma(-s, s, x); r = fma(e, 0.5*y, s); max(r, 0)
// against hipcc's IEEE sqrtf (correctly rounded). Prints mismatch counts and
// examples. Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 sqrt_rsq_probe.hip -o sqrt_rsq_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int M>
__device__ __forceinline__ float cand(float x)
{
    if constexpr (M == 0) {
        const float y = __builtin_amdgcn_rsqf(x);
        const float s = x * y, h = 0.5f * y;
        const float e = __builtin_fmaf(-s, s, x);
        return __builtin_fmaxf(__builtin_fmaf(e, h, s), 0.0f);
    } else {
        const float s = __builtin_amdgcn_sqrtf(x);
        const float y = __builtin_amdgcn_rsqf(x);
        const float e = __builtin_fmaf(-s, s, x);
        return __builtin_fmaxf(__builtin_fmaf(e, 0.5f * y, s), 0.0f);
    }
}

template <int M>
__global__ void probe(uint32_t base, unsigned long long *cnt, uint32_t *ex)
{
    const uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float(u);
    if (!((x >= 0x1p-96f && x <= 0x1p96f) || u == 0u)) return;
    const float a = cand<M>(x);
    const float b = __builtin_sqrtf(x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
        const unsigned long long k = atomicAdd(cnt, 1ull);
        if (k < 8) ex[k] = u;
    }
}

template <int M>
static void run(const char *name)
{
    unsigned long long *cnt;
    uint32_t *ex;
    hipMalloc(&cnt, 8);
    hipMalloc(&ex, 32);
    hipMemset(cnt, 0, 8);
    hipMemset(ex, 0, 32);
    const uint32_t chunk = 1u << 28;
    for (uint64_t b = 0; b <= 0x7f7fffffull; b += chunk)
        hipLaunchKernelGGL(probe<M>, dim3(chunk / 256), dim3(256), 0, 0, (uint32_t)b, cnt, ex);
    unsigned long long h = 0;
    uint32_t he[8];
    hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost);
    hipMemcpy(he, ex, 32, hipMemcpyDeviceToHost);
    printf("%s: %llu mismatches in [2^-96, 2^96] and 0\n", name, h);
    for (unsigned long long i = 0; i < h && i < 8; ++i) {
        const float x = *(float *)&he[i];
        printf("  x bits 0x%08x (%g)\n", he[i], x);
    }
    hipFree(cnt);
    hipFree(ex);
}

int main()
{
    run<0>("A rsq, x*y, one correction");
    run<1>("B sqrt + rsq, one correction");
    printf("hip: %s\n", hipGetErrorString(hipDeviceSynchronize()));
    return 0;
}
