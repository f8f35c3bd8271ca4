// VALU issue rate on gfx950 against waves per SIMD: a grid of exactly W waves
// on every SIMD (256 CUs x 4 SIMDs, one workgroup of 4 waves per CU per W),
// each wave running N iterations of
//   fma8   8 independent v_fma_f32 chains,
//   fma1   one dependent v_fma_f32 chain,
//   trans  4 independent v_sqrt_f32 / v_rcp_f32 chains,
//   pair   the step kernel's FAST pair math (pair_dist<true> + pair_angle<true>)
//          on 4 independent pairs per iteration,
// timed with hipEvents over the whole grid. Prints cycles per VALU
// instruction per SIMD (at the clock given on the command line, default 2.4).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 valu_rate.hip -o valu_rate
#include "../../marl-nav_amd/csrc/marlnav_step.hip"

namespace probe {

template <int MODE>
__global__ void __launch_bounds__(256) run(int iters, float *out, float seed)
{
    const float l = (float)threadIdx.x * 1e-3f + seed;
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = l + (float)i;
    float acc = 0.0f;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0) {  // 8 independent fma chains: 8 VALU
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) a[i] = __builtin_fmaf(a[i], 0.999f, 1e-3f);
        } else if constexpr (MODE == 1) {  // one dependent chain: 32 VALU
#pragma unroll
            for (int r = 0; r < 32; ++r) a[0] = __builtin_fmaf(a[0], 0.999f, 1e-3f);
        } else if constexpr (MODE == 2) {  // 4 independent sqrt + 4 rcp: 8 trans
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = __builtin_amdgcn_sqrtf(a[i]);
#pragma unroll
            for (int i = 4; i < 8; ++i) a[i] = __builtin_amdgcn_rcpf(a[i]);
        } else {  // 4 pairs of the FAST pair math
            bool ok = true;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float d = pair_dist<true>(a[4], a[5], a[i], a[i + 4], ok);
                const float g = pair_angle<true>(a[4], a[5], a[i], a[i + 4], 0.6f, 0.8f, d, 0.1f, ok);
                acc += d + g;
                a[i] = a[i] + 1e-3f;
            }
            asm volatile("" : "+v"(acc));
        }
    }
    float s = acc;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i];
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (s == 12345.678f) out[threadIdx.x] = s;  // keep the work
    if (blockIdx.x == 0 && threadIdx.x == 0) out[1023] = (float)(c1 - c0) / (float)iters;
}

}  // namespace probe

static float g_cyc;
template <int MODE>
static double time_mode(int W, int iters)
{
    float *out;
    hipMalloc(&out, 1024 * 4);
    const dim3 grid(256 * W), block(256);  // 4 waves per block: one per SIMD
    hipLaunchKernelGGL(probe::run<MODE>, grid, block, 0, 0, iters, out, 1.0f);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(probe::run<MODE>, grid, block, 0, 0, iters, out, 1.0f);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, e0, e1);
    float cyc = 0.0f;
    hipMemcpy(&cyc, out + 1023, 4, hipMemcpyDeviceToHost);
    g_cyc = cyc;
    hipFree(out);
    return ms * 1e-3 / 5.0;
}

int main(int argc, char **argv)
{
    const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
    // VALU instructions per iteration counted from the ISA of each mode (read
    // off by the caller; printed here as seconds per iteration per wave)
    const int iters = 20000;
    for (int W = 1; W <= 8; W *= 2) {
        for (int W2 : {W, W == 2 ? 3 : 0}) {
            if (W2 == 0) continue;
            float c[4];
            const double t0 = time_mode<0>(W2, iters); c[0] = g_cyc;
            const double t1 = time_mode<1>(W2, iters); c[1] = g_cyc;
            const double t2 = time_mode<2>(W2, iters); c[2] = g_cyc;
            const double t3 = time_mode<3>(W2, iters / 10); c[3] = g_cyc;
            const double cyc = ghz * 1e9 / iters;
            printf("waves/SIMD %d: cycles per iteration at %.1f GHz (wall) | s_memtime of one wave: "
                   "fma8x4 %.1f|%.1f  fma1x32 %.1f|%.1f  trans8 %.1f|%.1f  pair4 %.1f|%.1f\n",
                   W2, ghz, t0 * cyc, c[0], t1 * cyc, c[1], t2 * cyc, c[2], t3 * cyc * 10, c[3]);
        }
    }
    printf("hip: %s\n", hipGetErrorString(hipDeviceSynchronize()));
    return 0;
}
