// Issue cost of single VALU instruction forms on gfx950 at 8 waves per SIMD
// (256 CUs x 4 SIMDs x 8): each wave runs ITERS x 8 independent copies of one
// instruction (inline asm, 8 accumulators), timed with hipEvents over the grid.
// Prints SIMD cycles per wave-instruction at the given clock (default 2.4 GHz).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 valu_cost.hip -o valu_cost
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int M>
__global__ void __launch_bounds__(256) run(int iters, float *out, float seed, uint64_t m, float bs)
{
    typedef float v2 __attribute__((ext_vector_type(2)));
    float a[8], b = seed * 0.5f + 1.0f;
    double d[8], db = (double)seed * 0.25 + 1.0;
    for (int i = 0; i < 8; ++i) d[i] = (double)seed + (double)(threadIdx.x + i);
    v2 pa[8], pb = v2{b, b};
    for (int i = 0; i < 8; ++i) pa[i] = v2{seed + (float)i, seed - (float)threadIdx.x};
    for (int i = 0; i < 8; ++i) a[i] = seed + (float)(threadIdx.x + i);

    for (int it = 0; it < iters; ++it) {
#define OP(i)                                                                                         \
    if constexpr (M == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));             \
    if constexpr (M == 1) asm volatile("v_fmaak_f32 %0, %0, %1, 0x3f7ff972" : "+v"(a[i]) : "v"(b));  \
    if constexpr (M == 2) asm volatile("v_mul_f32_e32 %0, 0x3f7ff972, %0" : "+v"(a[i]));             \
    if constexpr (M == 3) asm volatile("v_max_f32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b));           \
    if constexpr (M == 4) asm volatile("v_med3_f32 %0, %0, %1, 1.0" : "+v"(a[i]) : "v"(b));         \
    if constexpr (M == 5) asm volatile("v_add_u32_e32 %0, 1, %0" : "+v"(a[i]));                      \
    if constexpr (M == 6) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(m)); \
    if constexpr (M == 7) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));  \
    if constexpr (M == 8) {                                                                           \
        uint64_t c;                                                                                   \
        asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(c) : "v"(a[i]), "v"(b));                   \
        asm volatile("" ::"s"(c));                                                                    \
    }                                                                                                 \
    if constexpr (M == 9) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1" ::"v"(a[i]), "v"(b) : "vcc");  \
    if constexpr (M == 10) asm volatile("v_sqrt_f32_e32 %0, %0" : "+v"(a[i]));                       \
    if constexpr (M == 11) asm volatile("v_rcp_f32_e32 %0, %0" : "+v"(a[i]));                        \
    if constexpr (M == 12) asm volatile("v_fma_f32 %0, |%0|, -0.5, 0.5" : "+v"(a[i]));               \
    if constexpr (M == 13) asm volatile("v_sub_f32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b));          \
    if constexpr (M == 14) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "s"(bs), "v"(b)); \
    if constexpr (M == 15) asm volatile("v_cmp_gt_f32_e64 vcc, %0, %1" ::"v"(a[i]), "v"(b) : "vcc"); \
    if constexpr (M == 16) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(pa[i]) : "v"(pb)); \
    if constexpr (M == 17) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 1) & 7]));  \
    if constexpr (M == 18) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(d[i]) : "v"(a[i]), "v"(b) : "s0", "s1"); \
    if constexpr (M == 19) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(db));        \
    if constexpr (M == 20) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));           \
    if constexpr (M == 21) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));           \
    if constexpr (M == 22) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b));      \
    if constexpr (M == 23) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b));          \
    if constexpr (M == 24) asm volatile("v_alignbit_b32 %0, %0, %0, 13" : "+v"(a[i]));              \
    if constexpr (M == 25) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(db));
        REP8(OP)
#undef OP
    }
    float s = 0.0f;
    for (int i = 0; i < 8; ++i) s += a[i] + pa[i].x + pa[i].y + (float)d[i];
    if (s == 12345.678f) out[threadIdx.x] = s;
}

static const char *kNames[] = {"v_fma_f32 vvv", "v_fmaak_f32 (literal)", "v_mul_f32 literal",
                               "v_max_f32", "v_med3_f32", "v_add_u32", "v_cndmask_e64 sgpr",
                               "v_cndmask_e32 vcc", "v_cmp_gt_e64 ->sgpr", "v_cmp_gt_e32 ->vcc",
                               "v_sqrt_f32", "v_rcp_f32", "v_fma_f32 |x| consts",
                               "v_sub_f32", "v_fma_f32 sgpr operand", "v_cmp_gt_e64 ->vcc",
                               "v_pk_fma_f32", "v_mov_b32", "v_mad_u64_u32", "v_fma_f64",
                               "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24", "v_xor_b32",
                               "v_alignbit_b32", "v_mul_f64"};

template <int M>
static double t_mode(int W, int iters, float *out)
{
    const dim3 grid(256 * W), block(256);
    hipLaunchKernelGGL(run<M>, grid, block, 0, 0, iters, out, 1.0f, 0x5555555555555555ull, 0.25f);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(run<M>, grid, block, 0, 0, iters, out, 1.0f, 0x5555555555555555ull, 0.25f);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e-3 / 3.0;
}

template <int M>
static void report(double ghz, float *out)
{
    const int iters = 20000, W = 8;
    const double t = t_mode<M>(W, iters, out);
    printf("%-26s %.2f cycles per wave-instruction per SIMD\n", kNames[M],
           t * ghz * 1e9 / ((double)iters * 8 * W));
}

int main(int argc, char **argv)
{
    const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
    float *out;
    hipMalloc(&out, 1024 * 4);
    report<0>(ghz, out); report<1>(ghz, out); report<2>(ghz, out); report<3>(ghz, out);
    report<4>(ghz, out); report<5>(ghz, out); report<6>(ghz, out); report<7>(ghz, out);
    report<8>(ghz, out); report<9>(ghz, out); report<10>(ghz, out); report<11>(ghz, out);
    report<12>(ghz, out); report<13>(ghz, out); report<14>(ghz, out); report<15>(ghz, out);
    report<16>(ghz, out); report<17>(ghz, out);
    report<18>(ghz, out); report<19>(ghz, out); report<20>(ghz, out); report<21>(ghz, out);
    report<22>(ghz, out); report<23>(ghz, out); report<24>(ghz, out); report<25>(ghz, out);
    printf("hip: %s\n", hipGetErrorString(hipDeviceSynchronize()));
    return 0;
}
