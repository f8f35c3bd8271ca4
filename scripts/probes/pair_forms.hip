// The observe phase's pair math by instruction form:
//   scalar  the product's FAST pair math (pair_dist<true> + pair_angle<true>),
//           one pair per VALU instruction;
//   packed  pairs_fast<NP>: two pairs of a row per v_pk_add/mul/fma_f32
//           (pair2_fast), the per-element steps (rsq/rcp/sqrt, max/med3,
//           compares, selects) per element;
// on rows of 6 pairs (A3/O3: target, 3 obstacles, 2 agents) and 12 (an
// A16/O32 LPR-4 lane's slots), timed over a grid of exactly Wv waves on
// every SIMD (256 CUs x 4 SIMDs) with hipEvents and s_memtime, Wv = 1..8.
// Then an exactness check: scalar against pairs_fast<2> and <4> on 2^28
// random pair sets (coordinates of the fast range, headings on the unit
// circle, a cap that some pairs fall under, coincident points) must agree
// bit for bit on every distance and bearing.
// Build: make -C scripts/probes pair_forms   (same flags as the product)
#include "../../marl-nav_amd/csrc/marlnav_step.hip"

namespace probe {

// W = 0: the scalar pair math; else pairs_fast<NP> (two pairs per pair2_fast)
template <int NP, int W>
__global__ void __launch_bounds__(256) run(int iters, float *out, float seed)
{
    const float l = (float)threadIdx.x * 1e-3f + seed;
    float px[NP], py[NP], pd[NP], pg[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        px[i] = l + 0.37f * (float)i;
        py[i] = 0.5f * l - 0.21f * (float)i;
    }
    const float ox = 0.25f * l, oy = 1.0f - l, dirx = 0.6f, diry = 0.8f;
    float acc = 0.0f;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (W == 0) {
            bool ok = true;
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                pd[i] = pair_dist<true>(ox, oy, px[i], py[i], ok);
                pg[i] = pair_angle<true>(ox, oy, px[i], py[i], dirx, diry, pd[i], 0.1f, ok);
            }
        } else {
            pairs_fast<NP>(ox, oy, dirx, diry, px, py, 0.1f, pd, pg);
        }
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            acc += pd[i] + pg[i];
            px[i] = px[i] + 1e-3f;
        }
        asm volatile("" : "+v"(acc));
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (acc == 12345.678f) out[threadIdx.x] = acc;  // keep the work
    if (blockIdx.x == 0 && threadIdx.x == 0) out[1023] = (float)(c1 - c0) / (float)iters;
}

// exactness: scalar vs packed on n pair sets from a counter hash
__device__ __forceinline__ float uni(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return (float)(x >> 8) * 0x1p-24f;
}

__device__ __forceinline__ bool neq(float a, float b) { return __float_as_uint(a) != __float_as_uint(b); }

__global__ void __launch_bounds__(256) check(uint64_t n, unsigned long long *bad, uint32_t *ex)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long nb = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t k = (uint32_t)(i * 8u);
        // mostly O(1..10) coordinates, every 16th set at a wide scale
        const float sc = (i & 15) == 0 ? 0x1p12f * uni(k + 7u) + 0x1p-10f : 8.0f;
        const float ox = sc * (uni(k) - 0.5f), oy = sc * (uni(k + 1u) - 0.5f);
        const float px0 = ox + sc * (uni(k + 2u) - 0.5f) * ((i & 7) == 3 ? 0x1p-12f : 1.0f);
        const float py0 = oy + sc * (uni(k + 3u) - 0.5f);
        float px1 = (i & 31) == 5 ? ox : sc * (uni(k + 4u) - 0.5f);  // some coincident x
        float py1 = (i & 63) == 9 ? oy : sc * (uni(k + 5u) - 0.5f);
        if ((i & 127) == 17) { px1 = ox; py1 = oy; }                 // coincident points
        const float th = 6.2831853f * uni(k + 6u);
        const float dirx = cosf(th), diry = sinf(th);
        const float cap = 0.1f;
        const float qx[4] = {px0, px1, px1, px0}, qy[4] = {py0, py1, py0, py1};
        float ds[4], gs[4], d4[4], g4[4], d2[2], g2[2];
        bool unused = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ds[j] = pair_dist<true>(ox, oy, qx[j], qy[j], unused);
            gs[j] = pair_angle<true>(ox, oy, qx[j], qy[j], dirx, diry, ds[j], cap, unused);
        }
        pairs_fast<4>(ox, oy, dirx, diry, qx, qy, cap, d4, g4);
        pairs_fast<2>(ox, oy, dirx, diry, reinterpret_cast<const float(&)[2]>(qx),
                         reinterpret_cast<const float(&)[2]>(qy), cap, d2, g2);
        bool diff = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) diff = diff || neq(d4[j], ds[j]) || neq(g4[j], gs[j]);
#pragma unroll
        for (int j = 0; j < 2; ++j) diff = diff || neq(d2[j], ds[j]) || neq(g2[j], gs[j]);
        if (diff) {
            ++nb;
            if (atomicAdd(ex, 1u) < 4u)
                printf("mismatch i=%llu o=(%a,%a) p0=(%a,%a) p1=(%a,%a) dir=(%a,%a): scalar d=(%a,%a) "
                       "g=(%a,%a) packed4 d=(%a,%a) g=(%a,%a)\n",
                       (unsigned long long)i, ox, oy, px0, py0, px1, py1, dirx, diry, ds[0], ds[1],
                       gs[0], gs[1], d4[0], d4[1], g4[0], g4[1]);
        }
    }
    if (nb) atomicAdd(bad, nb);
}

}  // namespace probe

static float g_cyc;
template <int NP, int W>
static double time_mode(int Wv, int iters)
{
    float *out;
    (void)hipMalloc(&out, 1024 * 4);
    const dim3 grid(256 * Wv), block(256);  // 4 waves per block: one per SIMD
    hipLaunchKernelGGL((probe::run<NP, W>), grid, block, 0, 0, iters, out, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL((probe::run<NP, W>), grid, block, 0, 0, iters, out, 1.0f);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    float cyc = 0.0f;
    (void)hipMemcpy(&cyc, out + 1023, 4, hipMemcpyDeviceToHost);
    g_cyc = cyc;
    (void)hipFree(out);
    return ms * 1e-3 / 5.0;
}

template <int NP, int W>
static void row(int Wv, int iters, double ghz, double t_ref)
{
    const double t = time_mode<NP, W>(Wv, iters);
    const double cyc = ghz * 1e9 / iters;
    printf("  %2d pairs, %s W=%d: %7.1f cycles per wave-iteration (wall) | %7.1f s_memtime | vs scalar %.3f\n",
           NP, W ? "packed" : "scalar", W, t * cyc / Wv, g_cyc, t_ref > 0 ? t / t_ref : 1.0);
}

int main(int argc, char **argv)
{
    const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
    const uint64_t n = argc > 2 ? strtoull(argv[2], nullptr, 0) : (1ull << 28);
    const int iters = 4000;
    printf("# pair math per row iteration: wall cycles at %.1f GHz per wave (grid time / waves per SIMD), "
           "s_memtime of one wave\n", ghz);
    for (int Wv : {1, 2, 3, 4, 8}) {
        printf("waves/SIMD %d\n", Wv);
        const double s6 = time_mode<6, 0>(Wv, iters);
        row<6, 0>(Wv, iters, ghz, s6);
        row<6, 2>(Wv, iters, ghz, s6);
        const double s12 = time_mode<12, 0>(Wv, iters / 2);
        row<12, 0>(Wv, iters / 2, ghz, s12);
        row<12, 2>(Wv, iters / 2, ghz, s12);
    }
    unsigned long long *bad;
    uint32_t *ex;
    (void)hipMalloc(&bad, 8);
    (void)hipMalloc(&ex, 4);
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(ex, 0, 4);
    hipLaunchKernelGGL(probe::check, dim3(4096), dim3(256), 0, 0, n, bad, ex);
    unsigned long long nb = 0;
    (void)hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
    printf("exactness: %llu of %llu pair sets differ between scalar and packed (pairs_fast<2>, <4>)\n", nb,
           (unsigned long long)n);
    printf("hip: %s\n", hipGetErrorString(hipDeviceSynchronize()));
    return 0;
}
