// Bit-exactness of the step kernel's fast fp32 paths against the IEEE
// (hipcc default) operations, on the GPU: sqrt_fast, div2_fast, div_c and
// recip_fast from marl-nav_amd/csrc/marlnav_step.hip, over random operands
// whose exponents sweep each guard's whole range and beyond. A sample counts
// only when the fast path's guard accepts it (`ok`); rejected samples take
// the IEEE redo in the kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 fastmath_probe.hip
#include "../../marl-nav_amd/csrc/marlnav_step.hip"

namespace probe {

__device__ uint32_t hash(uint64_t x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}

// random float with unbiased exponent uniform in [lo, hi], random mantissa, +sign
__device__ float rexp(uint32_t h1, uint32_t h2, int lo, int hi)
{
    const int e = lo + (int)(h1 % (uint32_t)(hi - lo + 1));
    return __uint_as_float(((uint32_t)(e + 127) << 23) | (h2 & 0x7FFFFFu));
}

__global__ void run(uint64_t seed, uint64_t n, unsigned long long *cnt, float *ex)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t base = seed * 0x9E3779B97F4A7C15ull + 8 * i;
        const uint32_t h[6] = {hash(base), hash(base + 1), hash(base + 2), hash(base + 3),
                               hash(base + 4), hash(base + 5)};
        const int test = (int)(i & 3);
        bool ok = true, bad = false;
        float a0 = 0, a1 = 0, a2 = 0;
        if (test == 0) {  // sqrt_fast
            const float x = rexp(h[0], h[1], -100, 100);
            const float s = sqrt_fast(x, ok);
            bad = __float_as_uint(s) != __float_as_uint(__builtin_sqrtf(x));
            a0 = x;
        } else if (test == 1) {  // div2_fast: |x|, |y| <= den
            const float den = rexp(h[0], h[1], -62, 62);
            const int sh = (int)(h[2] % 80);  // numerators down to den * 2^-80
            const float x = den * __uint_as_float(((uint32_t)(127 - sh) << 23) | (h[3] & 0x7FFFFFu)) * 0.5f *
                            ((h[4] & 1) ? -1.0f : 1.0f);
            const float y = den * ((float)(h[5] >> 8) * 0x1p-24f - 0.5f);
            float qx, qy;
            div2_fast(x, y, den, &qx, &qy, ok);
            bad = __float_as_uint(qx) != __float_as_uint(x / den) ||
                  __float_as_uint(qy) != __float_as_uint(y / den);
            a0 = x; a1 = y; a2 = den;
        } else if (test == 2) {  // div_c by a reward constant
            const float cs[8] = {3.0f, 1200.0f, 2.0f, 1.0f, 15.0f, 16.0f, 7.0f, 0.0f};
            float c = cs[h[0] & 7];
            if (c == 0.0f) c = rexp(h[1], h[2], -22, 22);
            const float x = rexp(h[3], h[4], -75, 75) * ((h[5] & 1) ? -1.0f : 1.0f);
            const DivC d = make_divc(c, ok);
            const float q = div_c(x, d, ok);
            bad = __float_as_uint(q) != __float_as_uint(x / c);
            a0 = x; a1 = c;
        } else {  // recip_fast on 1 + sd^2
            const float den = 1.0f + rexp(h[0], h[1], -30, 97);
            const float q = recip_fast(den, ok);
            bad = __float_as_uint(q) != __float_as_uint(1.0f / den);
            a0 = den;
        }
        if (ok) atomicAdd(&cnt[2 * test], 1ull);
        if (ok && bad) {
            const unsigned long long k = atomicAdd(&cnt[2 * test + 1], 1ull);
            if (k < 2) {
                float *e = ex + (test * 2 + k) * 3;
                e[0] = a0; e[1] = a1; e[2] = a2;
            }
        }
    }
}

}  // namespace probe

int main()
{
    unsigned long long *cnt;
    float *ex;
    hipMalloc(&cnt, 8 * 8);
    hipMalloc(&ex, 24 * 4);
    hipMemset(cnt, 0, 64);
    hipMemset(ex, 0, 96);
    const uint64_t n = 1ull << 31;
    for (int s = 0; s < 4; ++s)
        hipLaunchKernelGGL(probe::run, dim3(8192), dim3(256), 0, 0, (uint64_t)s + 11, n, cnt, ex);
    unsigned long long h[8];
    float e[24];
    hipMemcpy(h, cnt, 64, hipMemcpyDeviceToHost);
    hipMemcpy(e, ex, 96, hipMemcpyDeviceToHost);
    const char *names[4] = {"sqrt_fast", "div2_fast", "div_c", "recip_fast"};
    int fails = 0;
    for (int t = 0; t < 4; ++t) {
        printf("%-10s accepted %llu, mismatches %llu\n", names[t], h[2 * t], h[2 * t + 1]);
        for (int k = 0; k < 2 && k < (int)h[2 * t + 1]; ++k)
            printf("   e.g. %a %a %a\n", e[(t * 2 + k) * 3], e[(t * 2 + k) * 3 + 1], e[(t * 2 + k) * 3 + 2]);
        fails += h[2 * t + 1] != 0;
    }
    return fails;
}
