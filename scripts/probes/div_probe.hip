// Checks div2() (marl-nav_amd/csrc/marlnav_step.hip) against IEEE fp32
// division on the GPU: random operands over the ranges the step kernel sees
// (position differences up to 1e4 over distances 1e-12 .. 1e4) plus random
// bit patterns in the fast-path range. Build: hipcc --offload-arch=gfx950 -O3
// -ffp-contract=off div_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ void div2(float x, float y, float den, float *qx, float *qy)
{
    const bool sub = __builtin_amdgcn_classf(x, 0x90) | __builtin_amdgcn_classf(y, 0x90);
    if (!(den <= 0x1p96f) || sub) { *qx = x / den; *qy = y / den; return; }
    float r = __builtin_amdgcn_rcpf(den);
    r = __builtin_fmaf(__builtin_fmaf(-den, r, 1.0f), r, r);
    float q = x * r;
    q = __builtin_fmaf(__builtin_fmaf(-den, q, x), r, q);
    *qx = __builtin_fmaf(__builtin_fmaf(-den, q, x), r, q);
    q = y * r;
    q = __builtin_fmaf(__builtin_fmaf(-den, q, y), r, q);
    *qy = __builtin_fmaf(__builtin_fmaf(-den, q, y), r, q);
}

__device__ uint32_t hash(uint64_t x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}

__global__ void probe(uint64_t seed, uint64_t n, unsigned long long *bad, float *ex)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t h1 = hash(seed * 0x9E3779B97F4A7C15ull + 3 * i);
        const uint32_t h2 = hash(seed * 0x9E3779B97F4A7C15ull + 3 * i + 1);
        const uint32_t h3 = hash(seed * 0x9E3779B97F4A7C15ull + 3 * i + 2);
        // the kernel's domain: den = max(sqrt(fma(y, y, x*x)), 1e-12), so |x|, |y| <~ den
        const int mode = (int)(i % 4);
        const float ux = (float)(h1 >> 8) * 0x1p-24f - 0.5f, uy = (float)(h2 >> 8) * 0x1p-24f - 0.5f;
        float x, y;
        if (mode == 0) {        // positions up to 1e4 apart
            x = ux * 4000.0f; y = uy * 4000.0f;
        } else if (mode == 1) { // random exponents down to denormals
            const float sx = __uint_as_float(((uint32_t)(h3 % 254) << 23) | (h1 & 0x807FFFFFu));
            x = sx; y = uy * sx * 2.0f;
        } else if (mode == 2) { // tiny differences (clamped denominators)
            x = ux * 1e-11f; y = uy * 1e-11f;
        } else {                // huge magnitudes up to 2^96
            const float sc = __uint_as_float(((uint32_t)(127 + h3 % 97) << 23));
            x = ux * sc; y = uy * sc;
        }
        float d = __builtin_sqrtf(__builtin_fmaf(y, y, x * x));
        d = d > 1e-12f ? d : 1e-12f;
        float qx, qy;
        div2(x, y, d, &qx, &qy);
        const float rx = x / d, ry = y / d;
        if (__float_as_uint(qx) != __float_as_uint(rx) || __float_as_uint(qy) != __float_as_uint(ry)) {
            const unsigned long long k = atomicAdd(bad, 1ull);
            if (k < 4) { ex[3 * k] = x; ex[3 * k + 1] = y; ex[3 * k + 2] = d; }
        }
    }
}

int main()
{
    unsigned long long *bad;
    float *ex;
    hipMalloc(&bad, 8);
    hipMalloc(&ex, 64);
    hipMemset(bad, 0, 8);
    const uint64_t n = 1ull << 32;
    for (int s = 0; s < 4; ++s) hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, (uint64_t)s + 1, n, bad, ex);
    unsigned long long h = 0;
    float e[12] = {0};
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(e, ex, 48, hipMemcpyDeviceToHost);
    printf("div2 vs IEEE (kernel domain): %llu mismatches in %llu quotient pairs\n", h, 4ull * n);
    for (int k = 0; k < 4 && k < (int)h; ++k) printf("  x=%a y=%a d=%a\n", e[3 * k], e[3 * k + 1], e[3 * k + 2]);
    return h != 0;
}
