// (1) Exhaustive check of sqrtf(x) as (float)v_sqrt_f64((double)x) against
//     the IEEE correctly rounded sqrtf over every positive finite float (and
//     inside sqrt_fast's range [2^-96, 2^96]).
// (2) Issue cost of the three instructions at 8 waves per SIMD next to
//     v_fma_f32 (as scripts/probes/valu_cost.hip).
// Build: hipcc --offload-arch=gfx950 -O3 sqrt64_probe.hip -o sqrt64_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ float sqrt64(float x)
{
    double s;
    asm volatile("v_sqrt_f64 %0, %1" : "=v"(s) : "v"((double)x));
    return (float)s;
}

__global__ void check(uint32_t base, unsigned long long *cnt, unsigned long long *cnt_fast,
                      uint32_t *ex)
{
    const uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;
    if (u > 0x7f7fffffu) return;
    const float x = __uint_as_float(u);
    const float a = sqrt64(x), b = __builtin_sqrtf(x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
        const unsigned long long k = atomicAdd(cnt, 1ull);
        if (k < 8) ex[k] = u;
        if (x >= 0x1p-96f && x <= 0x1p96f) atomicAdd(cnt_fast, 1ull);
    }
}

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
template <int M>
__global__ void __launch_bounds__(256) cost(int iters, float *out, float seed)
{
    float a[8];
    double d[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = seed + (float)(threadIdx.x + i);
        d[i] = (double)a[i];
    }
    for (int it = 0; it < iters; ++it) {
#define OP(i)                                                                               \
    if constexpr (M == 0) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(a[i]));           \
    if constexpr (M == 1) asm volatile("v_cvt_f64_f32_e32 %0, %1" : "=v"(d[i]) : "v"(a[i])); \
    if constexpr (M == 2) asm volatile("v_sqrt_f64 %0, %0" : "+v"(d[i]));                  \
    if constexpr (M == 3) asm volatile("v_cvt_f32_f64_e32 %0, %1" : "=v"(a[i]) : "v"(d[i])); \
    if constexpr (M == 4) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[i]));
        REP8(OP)
#undef OP
    }
    float s = 0.0f;
    for (int i = 0; i < 8; ++i) s += a[i] + (float)d[i];
    if (s == 12345.678f) out[threadIdx.x] = s;
}

template <int M>
static void report(const char *name, float *out)
{
    const int iters = 20000, W = 8;
    const dim3 grid(256 * W), block(256);
    hipLaunchKernelGGL(cost<M>, grid, block, 0, 0, iters, out, 1.0f);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(cost<M>, grid, block, 0, 0, iters, out, 1.0f);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-22s %.2f cycles per wave-instruction per SIMD (2.4 GHz)\n", name,
           ms * 1e-3 / 3.0 * 2.4e9 / ((double)iters * 8 * W));
}

int main()
{
    unsigned long long *cnt, *cf;
    uint32_t *ex;
    float *out;
    hipMalloc(&cnt, 8);
    hipMalloc(&cf, 8);
    hipMalloc(&ex, 32);
    hipMalloc(&out, 4096);
    hipMemset(cnt, 0, 8);
    hipMemset(cf, 0, 8);
    const uint32_t chunk = 1u << 28;
    for (uint64_t b = 0; b <= 0x7f7fffffull; b += chunk)
        hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, (uint32_t)b, cnt, cf, ex);
    unsigned long long h = 0, hf = 0;
    uint32_t he[8] = {};
    hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hf, cf, 8, hipMemcpyDeviceToHost);
    hipMemcpy(he, ex, 32, hipMemcpyDeviceToHost);
    printf("(float)v_sqrt_f64((double)x) != IEEE sqrtf: %llu of 2139095040 positive finite floats; "
           "%llu inside [2^-96, 2^96]\n", h, hf);
    for (int i = 0; i < 8 && i < (int)h; ++i)
        printf("  x bits 0x%08x (%g)\n", he[i], (double)__builtin_bit_cast(float, he[i]));
    report<0>("v_fma_f32", out);
    report<1>("v_cvt_f64_f32", out);
    report<2>("v_sqrt_f64", out);
    report<3>("v_cvt_f32_f64", out);
    report<4>("v_sqrt_f32", out);
    printf("hip: %s\n", hipGetErrorString(hipDeviceSynchronize()));
    return 0;
}
