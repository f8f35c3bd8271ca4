// Exhaustive check of shorter fp32 division sequences against IEEE division
// (hipcc's correctly rounded x / d), over EVERY pair of significands: x and d
// in [1, 2), 2^23 x 2^23 pairs. Every step of the sequences below (v_rcp_f32,
// products, FMAs) commutes with scaling x and d by powers of two as long as
// no intermediate leaves the normal range - which the kernel's guards
// (div2_fast, div_c: |x|, d in [2^-60, 2^60]) ensure - and with signs, so
// the significand pairs decide every guarded case.
//   r0 = v_rcp_f32(d); r1 = r0 + r0 (1 - d r0)        (one Newton step)
//   R : r1 == RN(1/d)                                  (per d)
//   Q1: q = RN(x r1); q1 = q + r1 (x - d q)            (one correction)
//   Q2: q1 + r1 (x - d q1)                             (two: the shipped div2_fast)
// Counts the pairs where Q1 / Q2 differ from x / d, and the d where R fails.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 div_exhaustive.hip -o div_exhaustive
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__global__ void run(uint32_t d0, uint32_t nd, unsigned long long *cnt, uint32_t *ex)
{
    // one workgroup per d significand; its 256 threads sweep the 2^23 x
    const uint32_t dm = d0 + blockIdx.x;
    if (dm >= d0 + nd) return;
    const float d = __uint_as_float(0x3f800000u | dm);
    const float r0 = __builtin_amdgcn_rcpf(d);
    const float r1 = __builtin_fmaf(__builtin_fmaf(-d, r0, 1.0f), r0, r0);
    unsigned long long bad1 = 0, bad2 = 0;
    if (threadIdx.x == 0 && __float_as_uint(r1) != __float_as_uint(1.0f / d)) {
        atomicAdd(&cnt[0], 1ull);
        const unsigned long long k = atomicAdd(&cnt[3], 1ull);
        if (k < 16) { ex[4 * k] = 0; ex[4 * k + 1] = dm; ex[4 * k + 2] = __float_as_uint(r1); ex[4 * k + 3] = 0; }
    }
    for (uint32_t xm = threadIdx.x; xm < (1u << 23); xm += blockDim.x) {
        const float x = __uint_as_float(0x3f800000u | xm);
        const float ref = x / d;
        const float q = x * r1;
        const float q1 = __builtin_fmaf(__builtin_fmaf(-d, q, x), r1, q);
        const float q2 = __builtin_fmaf(__builtin_fmaf(-d, q1, x), r1, q1);
        const bool b1 = __float_as_uint(q1) != __float_as_uint(ref);
        const bool b2 = __float_as_uint(q2) != __float_as_uint(ref);
        bad1 += b1;
        bad2 += b2;
        if (b1 && bad1 == 1 && *(volatile unsigned long long *)&cnt[3] < 16) {
            const unsigned long long k = atomicAdd(&cnt[3], 1ull);
            if (k < 16) { ex[4 * k] = 1; ex[4 * k + 1] = dm; ex[4 * k + 2] = xm; ex[4 * k + 3] = __float_as_uint(q1); }
        }
    }
    // wave-reduce then one atomic per wave
    for (int o = 32; o > 0; o >>= 1) {
        bad1 += __shfl_xor(bad1, o);
        bad2 += __shfl_xor(bad2, o);
    }
    if ((threadIdx.x & 63) == 0) {
        if (bad1) atomicAdd(&cnt[1], bad1);
        if (bad2) atomicAdd(&cnt[2], bad2);
    }
}

int main(int argc, char **argv)
{
    const uint32_t total = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 0) : (1u << 23);
    const uint32_t chunk = 1u << 16;
    unsigned long long *cnt;
    uint32_t *ex;
    hipMalloc(&cnt, 4 * sizeof(unsigned long long));
    hipMalloc(&ex, 64 * sizeof(uint32_t));
    hipMemset(cnt, 0, 4 * sizeof(unsigned long long));
    unsigned long long h[4];
    for (uint32_t d0 = 0; d0 < total; d0 += chunk) {
        const uint32_t nd = total - d0 < chunk ? total - d0 : chunk;
        hipLaunchKernelGGL(run, dim3(nd), dim3(256), 0, 0, d0, nd, cnt, ex);
        if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "launch failed\n"); return 1; }
        if ((d0 / chunk) % 16 == 15 || d0 + nd >= total) {
            hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost);
            printf("d significands %u / %u: R fails %llu, Q1 fails %llu, Q2 fails %llu\n", d0 + nd, total,
                   h[0], h[1], h[2]);
            fflush(stdout);
        }
    }
    uint32_t e[64];
    hipMemcpy(e, ex, sizeof e, hipMemcpyDeviceToHost);
    const unsigned long long n = h[3] < 16 ? h[3] : 16;
    for (unsigned long long k = 0; k < n; ++k)
        printf("example %s d=0x%08x x=0x%08x got=0x%08x\n", e[4 * k] ? "Q1" : "R", 0x3f800000u | e[4 * k + 1],
               e[4 * k] ? 0x3f800000u | e[4 * k + 2] : e[4 * k + 2], e[4 * k + 3]);
    printf("pairs checked %llu\n", (unsigned long long)total << 23);
    return 0;
}
