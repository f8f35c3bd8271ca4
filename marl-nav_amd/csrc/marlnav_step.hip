// marlnav_step.hip - gfx950 (MI355X) kernels behind include/marlnav.h.
//
// One launch performs the whole Env.step of the reference
// (marlnav/environment.py:92-107): heading/speed integration, every
// agent->target/obstacle/agent distance and bearing, the reward terms, the
// terminal logic, the masked re-initialisation of finished envs and the
// recomputed observations of those envs.
//
// Three kernel families, one launch per step, picked on the host
// by shape and grid size (marlnav_step, end of file):
//   block_kernel  - one workgroup of A waves per 64 consecutive envs, lane =
//                   env, wave = agent (the compiled A3 shapes; the headline
//                   path), section "env-block kernel";
//   split_kernel  - LPR lanes per agent row, wave-private tiles (A16/O32, and
//                   small A3 grids), section "pair-split kernel";
//   wave_kernel   - generic runtime shapes.
// All stage their inputs in LDS with LDS-DMA, keep a lane's own row in
// registers, assemble the packed observation rows in LDS where they stream
// out with 16-byte stores, and re-initialise / re-observe only the envs that
// finished. No MFMA: nothing here contracts.
//
// Numerics: built with -ffp-contract=off and the HIP default
// correctly rounded fp32 division and sqrt, so every distance, dot product
// and reward term is the fp32 expression the reference's CPU path evaluates,
// summed in torch's order. sin/cos of the heading update are evaluated in
// double (sincos_k, identical code in oracle/marlnav_oracle.c) and rounded
// once; acos is the device libm's acosf.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/marlnav.h"

namespace {

constexpr float kPiF = 3.14159265358979323846f;
constexpr int kMaxAgents = 64;
constexpr int kMaxStride = 256;
constexpr int kWavesPerBlock = 4;
constexpr int kWaveLdsFloats = 4096;    // 16 KiB per wave, 64 KiB per block
constexpr int kObsTileMax = 2304;       // floats of packed obs staged per wave

// Timing-only ablation builds (scripts/kbench.py; never shipped, results
// wrong by construction): 1 no acos, 2 fp32 fast sin/cos, 4 fast division,
// 8 fast sqrt, 16 no observation math at all, 64 tile kernel returns at entry.
#ifndef MARLNAV_ABLATE
#define MARLNAV_ABLATE 0
#endif

// Diagnostic build (MARLNAV_STAMPS=1, scripts/kstamps.py): lane 0 of every
// wave records s_memrealtime / s_memtime at each phase boundary into a
// buffer registered with marlnav_debug_stamps().
#ifndef MARLNAV_STAMPS
#define MARLNAV_STAMPS 0
#endif
#if MARLNAV_STAMPS
__device__ unsigned long long *g_stamps;
#define STAMP(k)                                                                   \
    do {                                                                           \
        if (lane == 0) {                                                           \
            unsigned long long *sp_ = g_stamps + (size_t)gw * 24;                  \
            sp_[2 * (k)] = wall_clock64();                                         \
            sp_[2 * (k) + 1] = clock64();                                          \
        }                                                                          \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif

thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}
}  // namespace

// error reporting shared with the other translation units of the library
__attribute__((visibility("hidden"))) int marlnav_internal_fail(int code, const char *msg)
{
    return fail(code, "%s", msg);
}

namespace {

__host__ __device__ inline int obs_dim(int A, int O) { return 2 + 2 * O + 2 * (A - 1); }

// ------------------------------------------------------------- device math
__device__ __forceinline__ float clamp_t(float x, float lo, float hi)
{
    x = x < lo ? lo : x;  // NaN passes through like torch.clamp
    return x > hi ? hi : x;
}

// Observation rows and states of the env-block and pair-split kernels leave
// through streaming stores (`nt`): nothing in the launch reads them back, and
// dirty lines kept in the XCD's L2 only lengthen the end-of-launch
// write-back. Measured: 65536x3x3 10.3 -> 9.4 us, 65536x3x8 13.0 -> 11.5 us,
// 2^21 envs 150 -> 144 us, 4096x16x32 18.0 -> 17.3 us. Per-env scalars (one
// env per wave in the split kernel: 1-4 byte stores) measured slower with nt
// and stay plain, as do the tile/wave kernels' stores; MARLNAV_NT_STORES /
// MARLNAV_NT_OTHER switch the two groups.
#ifndef MARLNAV_NT_STORES
#define MARLNAV_NT_STORES 1
#endif
#ifndef MARLNAV_NT_OTHER
#define MARLNAV_NT_OTHER 0
#endif
constexpr bool kNtRows = MARLNAV_NT_STORES != 0;
constexpr bool kNtOther = MARLNAV_NT_OTHER != 0;
typedef float v4f_t __attribute__((ext_vector_type(4)));
typedef float v2f_t __attribute__((ext_vector_type(2)));

template <bool NT = kNtOther, class T>
__device__ __forceinline__ void out_st(T *p, T v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template <bool NT = kNtOther>
__device__ __forceinline__ void out_st4(float *p, float4 v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v4f_t{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f_t *>(p));
    else
        *reinterpret_cast<float4 *>(p) = v;
}

template <bool NT = kNtOther>
__device__ __forceinline__ void out_st2(float *p, float2 v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v2f_t{v.x, v.y}, reinterpret_cast<v2f_t *>(p));
    else
        *reinterpret_cast<float2 *>(p) = v;
}

// Fast-path switches for the pair math in FAST mode: 1 = the shortened
// sequence (bit-exact inside its guard, scripts/probes/fastmath_probe.hip),
// 0 = the IEEE operation. The tile kernels enter FAST mode only for a wave
// whose every coordinate passed coords_in_range() (which implies every
// per-pair guard), so there the guards are dead code. Kernels that evaluate
// the guards per pair (wave/split kernels) were measured slower with them and
// run IEEE-only (kGuardedFast).
#ifndef MARLNAV_FM_SQRT
#define MARLNAV_FM_SQRT 1
#endif
#ifndef MARLNAV_FM_DIV2   // 2: exponent-range guard, 1: magnitude compares, 0: IEEE
#define MARLNAV_FM_DIV2 1
#endif
constexpr bool kGuardedFast = false;
#ifndef MARLNAV_FM_TERMS
#define MARLNAV_FM_TERMS 0
#endif
// Internal MarlnavParams.flags bit set by marlnav_step when every reward
// parameter lies inside the short division sequences' guards
// (terms_fast_params): the observe_row_own reward terms then use them in
// FAST (coordinate-checked) waves. Never set by callers (above the public
// MARLNAV_* flag bits).
constexpr uint32_t kTermsFastFlag = 1u << 30;

// x == 0 or x = m * 2^e with e in [-59, 62] (|x| in [2^-60, 2^62)); NaN and
// infinities pass (they also fail the denominators' guard)
__device__ __forceinline__ bool exp_ok(float x)
{
    return (unsigned)(__builtin_amdgcn_frexp_expf(x) + 59) <= 121u;
}

// |x| in [lo, hi] or x == 0
__device__ __forceinline__ bool mag_ok(float x, float lo, float hi)
{
    const float ax = fabsf(x);
    return (ax >= lo && ax <= hi) || x == 0.0f;
}

// A coordinate the fast pair math accepts without per-pair guards: zero or
// |c| in [2^-20, 2^40]. If every position a row uses satisfies it, every
// nonzero difference is >= 2^-43 and <= 2^41, so each pair's squared
// distance lies in [2^-86, 2^83] (sqrt_fast guard [2^-96, 2^96]), each
// distance in [1e-12 clamp, 2^42] and each numerator zero or in
// [2^-43, 2^41] (div2_fast guard [2^-60, 2^60]).
__device__ __forceinline__ bool coord_ok(float c) { return mag_ok(c, 0x1p-20f, 0x1p40f); }

// coord_ok over many values without per-value compares: |c| as bits is
// monotone for non-negative floats, so accumulate min(bits - 1) (0 wraps to
// the largest value: zero passes) and max(bits) (NaN and inf exceed 2^40),
// then compare once. Equal to AND over coord_ok.
struct CoordRange {
    uint32_t lo = 0xffffffffu, hi = 0u;
    __device__ void add(float c)
    {
        const uint32_t u = __float_as_uint(c) & 0x7fffffffu;
        lo = u - 1u < lo ? u - 1u : lo;
        hi = u > hi ? u : hi;
    }
    __device__ bool ok() const
    {
        return lo >= __float_as_uint(0x1p-20f) - 1u && hi <= __float_as_uint(0x1p40f);
    }
};

// coord_ok over a full tile's staged obstacle (NOB floats) and target (NTG)
// coordinates, spread over the wave's lanes
template <int NOB, int NTG>
__device__ __forceinline__ bool tile_coords_ok(const float *ob, const float *tg, unsigned lane)
{
    bool ok = true;
#pragma unroll
    for (int k = 0; k * 64 < NOB; ++k) {
        const int i = k * 64 + (int)lane;
        if ((k + 1) * 64 <= NOB || i < NOB) ok = ok && coord_ok(ob[i]);
    }
#pragma unroll
    for (int k = 0; k * 64 < NTG; ++k) {
        const int i = k * 64 + (int)lane;
        if ((k + 1) * 64 <= NTG || i < NTG) ok = ok && coord_ok(tg[i]);
    }
    return ok;
}

// Correctly rounded sqrt for x in [2^-96, 2^96] or x == 0: hipcc's own
// IEEE sequence (v_sqrt_f32, then the neighbour whose residual straddles x)
// without its input scaling and special-value class fix-up, which only act
// outside that range; `ok` is cleared outside it (the caller redoes the row
// with the full sequence).
__device__ __forceinline__ float sqrt_fast(float x, bool &ok)
{
    ok &= (x >= 0x1p-96f && x <= 0x1p96f) || x == 0.0f;
    float s = __builtin_amdgcn_sqrtf(x);
    const float s_dn = __int_as_float(__float_as_int(s) - 1);
    const float s_up = __int_as_float(__float_as_int(s) + 1);
    // x - s_dn*s with the sign on the float operand (a free source modifier;
    // negating the integer-built neighbour costs a v_xor per pair)
    const float r_dn = __builtin_fmaf(s_dn, -s, x);
    const float r_up = __builtin_fmaf(s_up, -s, x);
    s = r_dn <= 0.0f ? s_dn : s;
    return r_up > 0.0f ? s_up : s;
}

// torch.cdist direct path (environment.py:271-274)
template <bool FAST = false>
__device__ __forceinline__ float pair_dist(float ox, float oy, float px, float py, bool &ok)
{
    const float dx = px - ox, dy = py - oy;
#if MARLNAV_ABLATE & 8
    return __builtin_amdgcn_sqrtf(__builtin_fmaf(dy, dy, dx * dx));
#else
    if constexpr (FAST && MARLNAV_FM_SQRT)
        return sqrt_fast(__builtin_fmaf(dy, dy, dx * dx), ok);
    else
        return __builtin_sqrtf(__builtin_fmaf(dy, dy, dx * dx));
#endif
}

__device__ __forceinline__ float pair_dist(float ox, float oy, float px, float py)
{
    bool ok = true;
    return pair_dist<false>(ox, oy, px, py, ok);
}

// Division by a wave-uniform constant c (a reward parameter): the same
// core sequence as div2_fast with the reciprocal refined once per use site
// (uniform, so once per wave). Guard: c in [2^-20, 2^20], the numerator zero
// or in [2^-70, 2^70], so every intermediate stays normal; `ok` cleared
// otherwise.
struct DivC {
    float c, r;
};

__device__ __forceinline__ DivC make_divc(float c, bool &ok)
{
    const float ac = fabsf(c);
    ok &= ac >= 0x1p-20f && ac <= 0x1p20f;
    float r = __builtin_amdgcn_rcpf(c);
    r = __builtin_fmaf(__builtin_fmaf(-c, r, 1.0f), r, r);
    return DivC{c, r};
}

__device__ __forceinline__ float div_c(float x, DivC d, bool &ok)
{
    ok &= mag_ok(x, 0x1p-70f, 0x1p70f);
    float q = x * d.r;
    q = __builtin_fmaf(__builtin_fmaf(-d.c, q, x), d.r, q);
    return __builtin_fmaf(__builtin_fmaf(-d.c, q, x), d.r, q);
}

// 1 / den for den in [1, 2^96] (the bond term's 1 + sd^2): div2_fast's core.
__device__ __forceinline__ float recip_fast(float den, bool &ok)
{
    ok &= den <= 0x1p96f;
    float r = __builtin_amdgcn_rcpf(den);
    r = __builtin_fmaf(__builtin_fmaf(-den, r, 1.0f), r, r);
    const float q = __builtin_fmaf(__builtin_fmaf(-den, r, 1.0f), r, r);
    return __builtin_fmaf(__builtin_fmaf(-den, q, 1.0f), r, q);
}

// Two correctly rounded quotients over one denominator. This is hipcc's own
// IEEE fp32 division sequence (reciprocal refined by one Newton step, two
// residual corrections) with the v_div_scale / v_div_fixup range steps
// dropped and the reciprocal shared. Those steps only matter when a quotient,
// reciprocal or residual leaves the normal range; the guard keeps every
// intermediate normal: den in [2^-60, 2^60] (den is a pair distance clamped
// at 1e-12, so |x|, |y| <= den) and numerators zero or >= 2^-60 in magnitude.
// `ok` is cleared otherwise and the caller redoes the row with IEEE division.
// Branch-free, so consecutive pairs interleave. Checked bit-exact against
// IEEE division on the GPU: scripts/probes/fastmath_probe.hip.
__device__ __forceinline__ void div2_fast(float x, float y, float den, float *qx, float *qy,
                                          bool &ok)
{
#if MARLNAV_FM_DIV2 == 2
    ok &= den >= 0x1p-60f && den <= 0x1p60f && exp_ok(x) && exp_ok(y);
#else
    ok &= den >= 0x1p-60f && den <= 0x1p60f && mag_ok(x, 0x1p-60f, 0x1p60f) &&
          mag_ok(y, 0x1p-60f, 0x1p60f);
#endif
    float r = __builtin_amdgcn_rcpf(den);
    r = __builtin_fmaf(__builtin_fmaf(-den, r, 1.0f), r, r);
    float q = x * r;
    q = __builtin_fmaf(__builtin_fmaf(-den, q, x), r, q);
    *qx = __builtin_fmaf(__builtin_fmaf(-den, q, x), r, q);
    q = y * r;
    q = __builtin_fmaf(__builtin_fmaf(-den, q, y), r, q);
    *qy = __builtin_fmaf(__builtin_fmaf(-den, q, y), r, q);
}

// _get_angles (environment.py:276-286) + the dist < 0.1 cap (:172-177).
// FAST: shared-reciprocal division (clears ok when it may differ from IEEE).
template <bool FAST = false>
__device__ __forceinline__ float pair_angle(float ox, float oy, float px, float py,
                                            float dirx, float diry, float dist, float cap,
                                            bool &ok)
{
    const float dx = px - ox, dy = py - oy;
    // F.normalize's clamp_min(1e-12). FAST (finite, non-negative dist): one
    // v_med3 instead of a canonicalize + v_max
    const float den = FAST ? __builtin_amdgcn_fmed3f(dist, 1e-12f, __builtin_inff())
                           : (dist > 1e-12f ? dist : 1e-12f);
#if MARLNAV_ABLATE & 4
    const float nx = __fdividef(dx, den), ny = __fdividef(dy, den);
#else
    float nx, ny;
    if constexpr (FAST && MARLNAV_FM_DIV2 != 0) {
        div2_fast(dx, dy, den, &nx, &ny, ok);
    } else {
        nx = dx / den;
        ny = dy / den;
    }
#endif
    float dot = dirx * nx + diry * ny;
    // FAST: dot is finite, so the clamp is one v_med3 (no compare/select
    // pairs and their VCC hazard nops); -0 passes through either way
    dot = FAST ? __builtin_amdgcn_fmed3f(dot, -1.0f, 1.0f) : clamp_t(dot, -1.0f, 1.0f);
    const float orth_x = nx - dot * dirx;
#if MARLNAV_ABLATE & 1
    const float ang = (orth_x > 0.0f ? -1.0f : 1.0f) * dot;
#else
    const float ang = (orth_x > 0.0f ? -1.0f : 1.0f) * acosf(dot);
#endif
    return dist < cap ? 0.0f : ang;
}

// sin/cos of an angle already clamped to [-pi, pi], evaluated in double and
// rounded once: Cody-Waite reduction by pi/2 (two-part constant, |k| <= 2)
// and the fdlibm __kernel_sin/__kernel_cos minimax polynomials on
// [-pi/4, pi/4]. Identical expression tree in oracle/marlnav_oracle.c.
__device__ __forceinline__ void sincos_k(float th, float *s_out, float *c_out)
{
#if MARLNAV_ABLATE & 2
    __sincosf(th, s_out, c_out);
#else
    const double x = (double)th;
    const double k = __builtin_rint(x * 6.36619772367581382433e-01);
    double r = __builtin_fma(-k, 1.57079632679489655800e+00, x);
    r = __builtin_fma(-k, 6.12323399573676603587e-17, r);
    r = k == 0.0 ? x : r;  // keeps the sign of -0
    const double z = r * r;
    double ps = __builtin_fma(1.58969099521155010221e-10, z, -2.50507602534068634195e-08);
    ps = __builtin_fma(ps, z, 2.75573137070700676789e-06);
    ps = __builtin_fma(ps, z, -1.98412698298579493134e-04);
    ps = __builtin_fma(ps, z, 8.33333333332248946124e-03);
    ps = __builtin_fma(ps, z, -1.66666666666666324348e-01);
    const double sn = r == 0.0 ? r : __builtin_fma(r * z, ps, r);  // sin(-0) = -0
    double pc = __builtin_fma(-1.13596475577881948265e-11, z, 2.08757232129817482790e-09);
    pc = __builtin_fma(pc, z, -2.75573143513906633035e-07);
    pc = __builtin_fma(pc, z, 2.48015872894767294178e-05);
    pc = __builtin_fma(pc, z, -1.38888888888741095749e-03);
    pc = __builtin_fma(pc, z, 4.16666666666666019037e-02);
    const double cs = __builtin_fma(z * z, pc, __builtin_fma(-0.5, z, 1.0));
    const int q = ((int)k) & 3;
    const double s = q == 0 ? sn : (q == 1 ? cs : (q == 2 ? -sn : -cs));
    const double c = q == 0 ? cs : (q == 1 ? -sn : (q == 2 ? -cs : sn));
    *s_out = (float)s;
    *c_out = (float)c;
#endif
}

// ----------------------------------------------------------- native RNG
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one v_mad_u64_u32 per product instead of v_mul_lo_u32 + v_mul_hi_u32
        const uint64_t p0 = (uint64_t)c[0] * 0xD2511F53u, p1 = (uint64_t)c[2] * 0xCD9E8D57u;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// uniform #idx of env gid at step s, in [0, 1) on a 24-bit grid
__device__ __forceinline__ float native_uniform(uint64_t seed, uint64_t gid, uint64_t s,
                                                uint32_t idx)
{
    uint32_t c[4] = {idx >> 2, (uint32_t)s, (uint32_t)gid,
                     (uint32_t)(gid >> 32) ^ ((uint32_t)(s >> 32) << 16)};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t r = c[idx & 3u];
    return (float)(r >> 8) * 0x1.0p-24f;
}

// _reinit_update (environment.py:86-90) for a finished env (mask 1):
// 0*old + 1*fresh, so a non-finite old value stays NaN. Idempotent in the
// old value (blend(blend(x, f), f) has blend(x, f)'s value), so readers that
// race with an in-place blend of the same element get the same number.
__device__ __forceinline__ float blend_in(float old, float fresh) { return 0.0f * old + fresh; }

// native TriangleIntitializer draw for one env (utils.py:375-398); BLEND:
// blended into the env's current values (a re-init), else written (the
// initial state)
template <bool NOISY, bool BLEND = true>
__device__ void native_fresh_env(int A, int S, const MarlnavParams &pr,
                                 const float *__restrict__ formation, uint64_t gid,
                                 uint64_t sidx, float *st, float *ob, float *tg)
{
    const auto put = [](float *d, float v) { *d = BLEND ? blend_in(*d, v) : v; };
    for (int j = 0; j < S; j += 2) {  // one Philox block = 2 obstacles
        uint32_t c[4] = {(uint32_t)(j >> 1), (uint32_t)sidx, (uint32_t)gid,
                         (uint32_t)(gid >> 32) ^ ((uint32_t)(sidx >> 32) << 16)};
        philox4x32_10(c, (uint32_t)pr.seed, (uint32_t)(pr.seed >> 32));
        put(ob + 2 * j, pr.obs_range_x * ((float)(c[0] >> 8) * 0x1.0p-24f - 0.5f) + pr.obs_mean_x);
        put(ob + 2 * j + 1, pr.obs_range_y * ((float)(c[1] >> 8) * 0x1.0p-24f - 0.5f) + pr.obs_mean_y);
        if (j + 1 < S) {
            put(ob + 2 * j + 2, pr.obs_range_x * ((float)(c[2] >> 8) * 0x1.0p-24f - 0.5f) + pr.obs_mean_x);
            put(ob + 2 * j + 3, pr.obs_range_y * ((float)(c[3] >> 8) * 0x1.0p-24f - 0.5f) + pr.obs_mean_y);
        }
    }
    put(tg, formation[5 * A]);
    put(tg + 1, formation[5 * A + 1]);
    for (int i = 0; i < A; ++i) {
        float f[5];
        for (int k = 0; k < 5; ++k) f[k] = formation[5 * i + k];
        if (NOISY) {
            const uint32_t base = (uint32_t)(2 * S);
            const float u1 = native_uniform(pr.seed, gid, sidx, base + 3 * i);
            const float u2 = native_uniform(pr.seed, gid, sidx, base + 3 * i + 1);
            const float u3 = native_uniform(pr.seed, gid, sidx, base + 3 * i + 2);
            const double rad = sqrt(-2.0 * log(1.0 - (double)u1));
            const double ang = 6.283185307179586 * (double)u2;
            const float z0 = (float)(rad * cos(ang)), z1 = (float)(rad * sin(ang));
            f[0] = f[0] + pr.ags_dist * (pr.noise_std * z0);
            f[1] = f[1] + pr.ags_dist * (pr.noise_std * z1);
            float sn, c;
            sincos_k(pr.angle_range * (u3 - 0.5f), &sn, &c);
            const float dx = f[2], dy = f[3];
            f[2] = c * dx + (-sn) * dy;
            f[3] = sn * dx + c * dy;
        }
        for (int k = 0; k < 5; ++k) put(st + 5 * i + k, f[k]);
    }
}

// torch's CPU float summation order over a contiguous row of n values
// (cascade_sum, aten/src/ATen/native/cpu/SumKernel.cpp; restated and pinned
// in oracle/marlnav_oracle.c: torch_row_sum). f maps each stored value.
template <typename F>
__device__ __forceinline__ float torch_row_sum(const float *x, int n, F f)
{
    if (n >= 8) {
        const int V = n >> 3, m = V >> 2;
        float acc[4][8];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[k][l] = 0.0f;
        for (int r = 0; r < m; ++r)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int l = 0; l < 8; ++l) acc[k][l] += f(x[(4 * r + k) * 8 + l]);
        for (int v = 4 * m; v < V; ++v)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[0][l] += f(x[v * 8 + l]);
#pragma unroll
        for (int k = 1; k < 4; ++k)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[0][l] += acc[k][l];
        float fin = 0.0f;
        for (int i = 8 * V; i < n; ++i) fin += f(x[i]);
#pragma unroll
        for (int l = 0; l < 8; ++l) fin += acc[0][l];
        return fin;
    }
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
    const int m = n >> 2;
    for (int r = 0; r < m; ++r) {
        a0 += f(x[4 * r]);
        a1 += f(x[4 * r + 1]);
        a2 += f(x[4 * r + 2]);
        a3 += f(x[4 * r + 3]);
    }
    for (int i = 4 * m; i < n; ++i) a0 += f(x[i]);
    a0 += a1;
    a0 += a2;
    a0 += a3;
    return a0;
}

// Make LDS writes of some lanes visible to later LDS reads of other lanes of
// the SAME wave: the LDS executes one wave's requests in issue order, so only
// the compiler must be kept from reordering across this point.
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------ wave staging
// Copy three contiguous global ranges into the wave's LDS slice with every
// global load issued before the first wait (a load -> LDS-store -> load loop
// would pay one memory round trip per iteration).
struct Span {
    const float *src;
    float *dst;
    int n;  // floats
};

__device__ __forceinline__ const float *span_src(const Span &a, const Span &b, const Span &c,
                                                 int i, int na, int nb)
{
    return i < na ? a.src + i : (i < na + nb ? b.src + (i - na) : c.src + (i - na - nb));
}

__device__ __forceinline__ float *span_dst(const Span &a, const Span &b, const Span &c, int i,
                                           int na, int nb)
{
    return i < na ? a.dst + i : (i < na + nb ? b.dst + (i - na) : c.dst + (i - na - nb));
}

// Load span x as 16-byte vectors, K per lane, branch-free: lanes past the end
// re-read the span's first vector (or, for a span shorter than one vector,
// the first vector of `safe`), so every load is in bounds and the loads issue
// back to back; the wait lands at the first LDS write.
template <int K>
__device__ __forceinline__ void load_vecs(const Span &x, const float *safe, int lane, float4 (&r)[K])
{
    const int n4 = x.n >> 2;
    const float4 *src = reinterpret_cast<const float4 *>(n4 > 0 ? x.src : safe);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = lane + 64 * k;
        r[k] = src[i < n4 ? i : 0];
    }
}

// Keep the compiler from sinking the loads of r next to their LDS stores:
// the values must be in VGPRs here, after every load of the tile was issued.
template <int K>
__device__ __forceinline__ void pin_vecs(float4 (&r)[K])
{
#pragma unroll
    for (int k = 0; k < K; ++k) asm volatile("" : "+v"(r[k].x), "+v"(r[k].y), "+v"(r[k].z), "+v"(r[k].w));
}

template <int K>
__device__ __forceinline__ void store_vecs(const Span &x, int lane, const float4 (&r)[K])
{
    const int n4 = x.n >> 2;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = lane + 64 * k;
        if (i < n4) reinterpret_cast<float4 *>(x.dst)[i] = r[k];
    }
    for (int i = lane + 64 * K; i < n4; i += 64)  // spans longer than K vectors per lane
        reinterpret_cast<float4 *>(x.dst)[i] = reinterpret_cast<const float4 *>(x.src)[i];
}

// Stage three spans into the wave's LDS slice. KA/KB/KC: vectors per lane
// loaded ahead for each span (exact for compile-time tile shapes).
template <int KA, int KB, int KC, bool ALIGNED>
__device__ __forceinline__ void stage_spans(Span a, Span b, Span c, int lane)
{
    const bool vec = ALIGNED || (((reinterpret_cast<uintptr_t>(a.src) |
                                   reinterpret_cast<uintptr_t>(b.src) |
                                   reinterpret_cast<uintptr_t>(c.src)) & 15u) == 0 && a.n >= 4);
    if (!vec) {  // unaligned tile base (only W < 4 tiles): plain copy
        const int nt = a.n + b.n + c.n;
        for (int i = lane; i < nt; i += 64)
            *span_dst(a, b, c, i, a.n, b.n) = *span_src(a, b, c, i, a.n, b.n);
        return;
    }
    float4 ra[KA], rb[KB], rc[KC];
    load_vecs<KA>(a, a.src, lane, ra);
    load_vecs<KB>(b, a.src, lane, rb);
    load_vecs<KC>(c, a.src, lane, rc);
    // scalar tails (< 4 floats per span, partial last tile only): lanes 0..11
    const int tw = lane >> 2, tj = lane & 3;
    const Span &tsp = tw == 0 ? a : (tw == 1 ? b : c);
    const bool has_tail = lane < 12 && tj < (tsp.n & 3);
    const int toff = (tsp.n & ~3) + tj;
    float t = has_tail ? tsp.src[toff] : 0.0f;
    pin_vecs<KA>(ra);
    pin_vecs<KB>(rb);
    pin_vecs<KC>(rc);
    asm volatile("" : "+v"(t));
    store_vecs<KA>(a, lane, ra);
    store_vecs<KB>(b, lane, rb);
    store_vecs<KC>(c, lane, rc);
    if (has_tail) tsp.dst[toff] = t;
}

// Stream n floats of the wave's LDS slice to global memory (16-byte stores
// when the destination allows), optionally also the ObsNormalizer output
// (utils.py:530-532) of every element.
__device__ __forceinline__ void wave_store(float *__restrict__ dst, const float *__restrict__ src,
                                           int n, int lane, float *__restrict__ nrm_dst,
                                           const float *__restrict__ mean,
                                           const float *__restrict__ scale, int D)
{
    int head = 0;
    if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
        const int n4 = n >> 2;
        for (int i = lane; i < n4; i += 64)
            out_st4(dst + 4 * i, *reinterpret_cast<const float4 *>(src + 4 * i));
        head = n4 << 2;
    }
    for (int i = head + lane; i < n; i += 64) out_st(dst + i, src[i]);
    if (nrm_dst) {
        for (int i = lane; i < n; i += 64) {
            const int k = i % D;
            nrm_dst[i] = (src[i] - mean[k]) / scale[k];
        }
    }
}

// ------------------------------------------------------------ row observe
struct RowOut {
    float r_miss, r_hit;  // agent reward if the env misses / reaches the target
    unsigned flags;       // bit0: obstacle or agent collision, bit1: in target
};

// observations() for agent row `a` of one env (environment.py:139-180), with
// the per-agent reward terms of _rews_and_terms (:184-269) when TERMS.
// `row` is the packed output row (LDS or global, stride 1).
template <int A_T, int O_T, bool TERMS>
__device__ __forceinline__ RowOut observe_row(int Arun, int Orun, const float *__restrict__ sts,
                                              const float *__restrict__ obe,
                                              const float *__restrict__ tge, int a,
                                              float *__restrict__ row, const MarlnavParams &pr)
{
    const int A = A_T ? A_T : Arun;
    const int O = O_T ? O_T : Orun;
    const float cap = pr.cap_distance;
    const float ox = sts[5 * a], oy = sts[5 * a + 1];
    const float dx = sts[5 * a + 2], dy = sts[5 * a + 3];

    const float tx = tge[0], ty = tge[1];
    const float td = pair_dist(ox, oy, tx, ty);
    bool ok = true;
    const float ta = pair_angle(ox, oy, tx, ty, dx, dy, td, cap, ok);
    row[0] = ta;
    row[1] = td;

    bool ob_risk = false, ob_col = false;
#pragma unroll
    for (int j = 0; j < O; ++j) {
        const float px = obe[2 * j], py = obe[2 * j + 1];
        const float d = pair_dist(ox, oy, px, py);
        row[2 + j] = pair_angle(ox, oy, px, py, dx, dy, d, cap, ok);
        row[2 + O + j] = d;
        if (TERMS) {
            ob_risk |= d < pr.ob_risk_dist;
            ob_col |= d < pr.ob_coll_dist;
        }
    }

    bool ag_risk = false, ag_col = false;
    float band = 0.0f;
    float *ang_out = row + 2 + 2 * O;
    float *dst_out = ang_out + (A - 1);
    int k = 0;
#pragma unroll
    for (int m = 0; m < A; ++m) {
        if (m == a) continue;
        const float px = sts[5 * m], py = sts[5 * m + 1];
        const float d = pair_dist(ox, oy, px, py);
        ang_out[k] = pair_angle(ox, oy, px, py, dx, dy, d, cap, ok);
        dst_out[k] = d;
        ++k;
        if (TERMS) {
            ag_risk |= d < pr.ag_risk_dist;
            ag_col |= d < pr.ag_coll_dist;
            band += (pr.agents_min_d < d && d < pr.agents_max_d) ? 1.0f : 0.0f;
        }
    }

    RowOut out{0.0f, 0.0f, 0u};
    if (TERMS) {
        const float head = fabsf(ta) < pr.max_angle_diff ? 1.0f : 0.0f;
        const float dsc = (band < pr.max_at_prop_d ? band : pr.max_at_prop_d) / pr.max_at_prop_d;
        const float soft = -1.0f * (td / pr.init_dist);
        // _bond_reward (environment.py:264-269), summed in torch's order over
        // the others_distances just written to this row
        const float ideal = pr.ideal_dist, sharp = pr.bond_sharpness;
        const float bond = torch_row_sum(dst_out, A - 1, [ideal, sharp](float d) {
            const float sd = (d - ideal) / sharp;
            return 1.0f / (1.0f + sd * sd);
        });
        const float bondm = bond / (float)(A - 1);
        const float risk = (ob_risk || ag_risk) ? 1.0f : 0.0f;
        float rm = pr.target_factor * 0.0f + pr.heading_factor * head;
        float rh = pr.target_factor * 1.0f + pr.heading_factor * head;
        rm = rm + pr.distance_factor * dsc;
        rh = rh + pr.distance_factor * dsc;
        rm = rm + pr.soft_factor * soft;
        rh = rh + pr.soft_factor * soft;
        rm = rm + pr.bond_factor * bondm;
        rh = rh + pr.bond_factor * bondm;
        rm = rm - pr.risk_factor * risk;
        rh = rh - pr.risk_factor * risk;
        out.r_miss = rm;
        out.r_hit = rh;
        out.flags = ((ob_col || ag_col) ? 1u : 0u) | ((td < pr.target_radius) ? 2u : 0u);
    }
    return out;
}

// torch_row_sum over N values held in registers (compile-time indices, so the
// array stays in VGPRs).
template <int N, typename F>
__device__ __forceinline__ float torch_row_sum_r(const float *x, F f)
{
    if constexpr (N >= 8) {
        constexpr int V = N / 8, M = V / 4;
        float acc[4][8];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[k][l] = 0.0f;
#pragma unroll
        for (int r = 0; r < M; ++r)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int l = 0; l < 8; ++l) acc[k][l] += f(x[(4 * r + k) * 8 + l]);
#pragma unroll
        for (int v = 4 * M; v < V; ++v)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[0][l] += f(x[v * 8 + l]);
#pragma unroll
        for (int k = 1; k < 4; ++k)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[0][l] += acc[k][l];
        float fin = 0.0f;
#pragma unroll
        for (int i = 8 * V; i < N; ++i) fin += f(x[i]);
#pragma unroll
        for (int l = 0; l < 8; ++l) fin += acc[0][l];
        return fin;
    } else {
        float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
        constexpr int M = N / 4;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            a0 += f(x[4 * r]);
            a1 += f(x[4 * r + 1]);
            a2 += f(x[4 * r + 2]);
            a3 += f(x[4 * r + 3]);
        }
#pragma unroll
        for (int i = 4 * M; i < N; ++i) a0 += f(x[i]);
        a0 += a1;
        a0 += a2;
        a0 += a3;
        return a0;
    }
}

// observe_row with compile-time shape and the packed row kept in registers
// (row[D]); others are visited as j = 0..A-2 -> agent j + (j >= a), so
// every row index is a compile-time constant.
// The own row (ox, oy, dx, dy) comes in registers; the env's other agents
// are read from sts.
template <int A, int O, bool TERMS, bool FAST>
__device__ __forceinline__ RowOut observe_row_own(const float *__restrict__ sts,
                                                  const float *__restrict__ obe,
                                                  const float *__restrict__ tge, int a,
                                                  float ox, float oy, float dx, float dy,
                                                  float *row, const MarlnavParams &pr, bool &ok)
{
    const float cap = pr.cap_distance;
    const float td = pair_dist<FAST>(ox, oy, tge[0], tge[1], ok);
    const float ta = pair_angle<FAST>(ox, oy, tge[0], tge[1], dx, dy, td, cap, ok);
    row[0] = ta;
    row[1] = td;
    bool ob_risk = false, ob_col = false;
#pragma unroll
    for (int j = 0; j < O; ++j) {
        const float px = obe[2 * j], py = obe[2 * j + 1];
        const float d = pair_dist<FAST>(ox, oy, px, py, ok);
        row[2 + j] = pair_angle<FAST>(ox, oy, px, py, dx, dy, d, cap, ok);
        row[2 + O + j] = d;
        if (TERMS) {
            ob_risk |= d < pr.ob_risk_dist;
            ob_col |= d < pr.ob_coll_dist;
        }
    }
    bool ag_risk = false, ag_col = false;
    float band = 0.0f;
#pragma unroll
    for (int j = 0; j < A - 1; ++j) {
        const int m = j + (j >= a ? 1 : 0);
        const float px = sts[5 * m], py = sts[5 * m + 1];
        const float d = pair_dist<FAST>(ox, oy, px, py, ok);
        row[2 + 2 * O + j] = pair_angle<FAST>(ox, oy, px, py, dx, dy, d, cap, ok);
        row[2 + 2 * O + (A - 1) + j] = d;
        if (TERMS) {
            ag_risk |= d < pr.ag_risk_dist;
            ag_col |= d < pr.ag_coll_dist;
            band += (pr.agents_min_d < d && d < pr.agents_max_d) ? 1.0f : 0.0f;
        }
    }
    RowOut out{0.0f, 0.0f, 0u};
    if (TERMS) {
        const float head = fabsf(ta) < pr.max_angle_diff ? 1.0f : 0.0f;
        const float ideal = pr.ideal_dist, sharp = pr.bond_sharpness;
        const float bandc = band < pr.max_at_prop_d ? band : pr.max_at_prop_d;
        float dsc, soft, bondm;
        if (FAST && (MARLNAV_FM_TERMS || (pr.flags & kTermsFastFlag))) {
            // exact: the host set kTermsFastFlag only for parameters inside
            // the div_c / recip_fast guards (terms_fast_params), and FAST
            // coordinates bound every distance (coord_ok), so every operand
            // below stays in range
            const DivC d_mapd = make_divc(pr.max_at_prop_d, ok);
            const DivC d_init = make_divc(pr.init_dist, ok);
            const DivC d_sharp = make_divc(sharp, ok);
            dsc = div_c(bandc, d_mapd, ok);
            soft = -1.0f * div_c(td, d_init, ok);
            const float bond = torch_row_sum_r<A - 1>(row + 2 + 2 * O + (A - 1), [&](float d) {
                const float sd = div_c(d - ideal, d_sharp, ok);
                return recip_fast(1.0f + sd * sd, ok);
            });
            bondm = bond / (float)(A - 1);  // the bond sum can be tiny: IEEE
        } else {
            dsc = bandc / pr.max_at_prop_d;
            soft = -1.0f * (td / pr.init_dist);
            const float bond = torch_row_sum_r<A - 1>(row + 2 + 2 * O + (A - 1), [ideal, sharp](float d) {
                const float sd = (d - ideal) / sharp;
                return 1.0f / (1.0f + sd * sd);
            });
            bondm = bond / (float)(A - 1);
        }
        const float risk = (ob_risk || ag_risk) ? 1.0f : 0.0f;
        float rm = pr.target_factor * 0.0f + pr.heading_factor * head;
        float rh = pr.target_factor * 1.0f + pr.heading_factor * head;
        rm = rm + pr.distance_factor * dsc;
        rh = rh + pr.distance_factor * dsc;
        rm = rm + pr.soft_factor * soft;
        rh = rh + pr.soft_factor * soft;
        rm = rm + pr.bond_factor * bondm;
        rh = rh + pr.bond_factor * bondm;
        rm = rm - pr.risk_factor * risk;
        rh = rh - pr.risk_factor * risk;
        out.r_miss = rm;
        out.r_hit = rh;
        out.flags = ((ob_col || ag_col) ? 1u : 0u) | ((td < pr.target_radius) ? 2u : 0u);
    }
    return out;
}

template <int A, int O, bool TERMS, bool FAST>
__device__ __forceinline__ RowOut observe_row_regs(const float *__restrict__ sts,
                                                   const float *__restrict__ obe,
                                                   const float *__restrict__ tge, int a,
                                                   float *row, const MarlnavParams &pr,
                                                   bool &ok)
{
    return observe_row_own<A, O, TERMS, FAST>(sts, obe, tge, a, sts[5 * a], sts[5 * a + 1],
                                              sts[5 * a + 2], sts[5 * a + 3], row, pr, ok);
}

// Store a register row of D floats with the widest aligned vector stores.
template <int D>
__device__ __forceinline__ void store_row(float *__restrict__ dst, const float *row)
{
    if constexpr (D % 4 == 0) {
#pragma unroll
        for (int k = 0; k < D; k += 4)
            out_st4(dst + k, make_float4(row[k], row[k + 1], row[k + 2], row[k + 3]));
    } else if constexpr (D % 2 == 0) {
#pragma unroll
        for (int k = 0; k < D; k += 2) out_st2(dst + k, make_float2(row[k], row[k + 1]));
    } else {
#pragma unroll
        for (int k = 0; k < D; ++k) out_st(dst + k, row[k]);
    }
}

// -------------------------------------------------------------- LDS plan
// Per-wave LDS slice, in floats, identical on host and device.
struct WavePlan {
    int W, A, O, S, D, obs_lds;
    int off_st, off_ob, off_tg, off_obs, off_rm, off_rh, off_fl, off_env, floats;
};

__host__ __device__ inline int align4(int n) { return (n + 3) & ~3; }  // floats -> 16 B

// packed obs rows kept in registers for compile-time shapes up to this D
constexpr int kRowRegsMaxD = 40;

__host__ __device__ constexpr int static_obs_dim(int A_T, int O_T)
{
    return (A_T > 0 && O_T > 0) ? 2 + 2 * O_T + 2 * (A_T - 1) : 0;
}

__host__ __device__ inline WavePlan make_plan(int W, int A, int O, int S, bool row_regs)
{
    WavePlan p;
    p.W = W;
    p.A = A;
    p.O = O;
    p.S = S;
    p.D = obs_dim(A, O);
    p.obs_lds = !row_regs && W * A * p.D <= kObsTileMax;
    int o = 0;
    p.off_st = o;  o += align4(W * A * 5);
    p.off_ob = o;  o += align4(W * S * 2);
    p.off_tg = o;  o += align4(W * 2);
    p.off_obs = o; o += p.obs_lds ? align4(W * A * p.D) : 0;
    p.off_rm = o;  o += 64;
    p.off_rh = o;  o += 64;
    p.off_fl = o;  o += 64;
    p.off_env = o; o += 64;
    p.floats = o;
    return p;
}

struct StepArgs {
    MarlnavStepBuffers b;
    int64_t P;
    int64_t env_offset;
    int64_t ntiles;
    int64_t waves;     // waves in the grid (= counter slots)
    uint64_t step_idx;
    int W, A, O, S;
};

// --------------------------------------------------------------- step kernel
template <int A_T, int O_T, bool OBS_ONLY, bool NOISY = false>
__global__ void __launch_bounds__(64 * kWavesPerBlock) wave_kernel(StepArgs args, MarlnavParams pr)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
#if MARLNAV_STAMPS
    unsigned long long t_entry;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_entry));
#endif
    const int A = A_T ? A_T : args.A;
    const int O = O_T ? O_T : args.O;
    const int S = args.S, W = args.W;
    constexpr int D_T = static_obs_dim(A_T, O_T);
    constexpr bool REGROW = D_T > 0 && D_T <= kRowRegsMaxD;
    const WavePlan wp = make_plan(W, A, O, S, REGROW);
    const int D = wp.D;
    const int lane = threadIdx.x & 63;
    // wave-uniform: keep the tile bookkeeping in SGPRs
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t gw = (int64_t)blockIdx.x * kWavesPerBlock + wib;
    float *wl = lds + wib * wp.floats;
    float *st = wl + wp.off_st;
    float *ob = wl + wp.off_ob;
    float *tg = wl + wp.off_tg;
    float *obs_t = wl + wp.off_obs;
    float *rmiss = wl + wp.off_rm;
    float *rhit = wl + wp.off_rh;
    unsigned *rfl = reinterpret_cast<unsigned *>(wl + wp.off_fl);
    unsigned *envbits = reinterpret_cast<unsigned *>(wl + wp.off_env);
    const MarlnavStepBuffers &b = args.b;
    const bool norm = !OBS_ONLY && (pr.flags & MARLNAV_WRITE_OBS_NORM) != 0;
    const int el = lane / A, a = lane - el * A;
    unsigned c_trunc = 0, c_col = 0, c_tar = 0;

#if MARLNAV_STAMPS && (MARLNAV_ABLATE & 32)
    if ((threadIdx.x & 63) == 0) {  // dispatch-only probe: entry stamp and out
        const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
        for (int k = 0; k < 16; ++k) g_stamps[w * 24 + k] = t_entry;
        g_stamps[w * 24 + 16] = t_entry;
        g_stamps[w * 24 + 18] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
    }
    return;
#endif
    // one tile per wave (a grid-stride loop here makes the compiler keep every
    // loop-invariant parameter live in registers: 160+ VGPRs instead of ~80)
    {
        const int64_t tile = gw;
        if (tile >= args.ntiles) return;
        STAMP(0);
        const int64_t e0 = tile * W;
        const int ne = (int)((args.P - e0) < W ? (args.P - e0) : W);
        const int nr = ne * A;
        const bool row_on = lane < nr;
        const bool env_on = lane < ne;

        // ---- stage the tile; every global load in flight before any wait
        // (branch-free: idle lanes re-read lane 0's element)
        float2 act = make_float2(0.0f, 0.0f);
        float step_num_in = 0.0f;
        uint8_t term_in = 0;
        if (!OBS_ONLY) {
            act = reinterpret_cast<const float2 *>(b.actions)[e0 * A + (row_on ? lane : 0)];
            step_num_in = b.step_num[e0 + (env_on ? lane : 0)];
            term_in = b.terminates[e0 + (env_on ? lane : 0)];
        }
        // vectors per lane for the compile-time tile shape (S == O for variants)
        constexpr int W_T = A_T ? ((64 / A_T) >= 4 ? (64 / A_T) & ~3 : 64 / A_T) : 0;
        constexpr int KA = W_T ? (W_T * A_T * 5 / 4 + 63) / 64 : 2;
        constexpr int KB = (W_T && O_T) ? (W_T * O_T * 2 / 4 + 63) / 64 : 2;
        constexpr int KC = W_T ? (W_T * 2 / 4 + 63) / 64 : 1;
        // 16-byte aligned tiles by construction when W_T % 4 == 0 and S == O
        // (torch allocations are 256-byte aligned; marlnav_step checks it)
        stage_spans<KA, KB, KC, (W_T % 4 == 0 && W_T > 0)>(Span{b.states + e0 * A * 5, st, nr * 5},
                                Span{b.obstacles + e0 * S * 2, ob, ne * S * 2},
                                Span{b.target + e0 * 2, tg, ne * 2}, lane);
        wave_sync();
        STAMP(1);

        // ---- _move_agents (environment.py:113-123), own row only
        if (!OBS_ONLY && row_on) {
            float a0 = act.x, a1 = act.y;
            if (pr.flags & MARLNAV_SCALE_ACTIONS) {  // ActionScaler (utils.py:546-547)
                a0 = pr.act_scale[0] * a0 + pr.act_mean[0];
                a1 = pr.act_scale[1] * a1 + pr.act_mean[1];
            }
            float *s = st + 5 * lane;
            float sn, c;
            sincos_k(clamp_t(a0, -kPiF, kPiF), &sn, &c);
            const float dx = s[2], dy = s[3];
            const float ndx = c * dx + (-sn) * dy;
            const float ndy = sn * dx + c * dy;
            const float v = clamp_t(s[4] + clamp_t(a1, pr.min_accel, pr.max_accel),
                                    pr.min_speed, pr.max_speed);
            s[0] = s[0] + ndx * v;
            s[1] = s[1] + ndy * v;
            s[2] = ndx;
            s[3] = ndy;
            s[4] = v;
        }
        wave_sync();
        STAMP(2);

        // ---- observations of the moved state + reward terms (:99-100)
        float *out_row = wp.obs_lds ? obs_t + lane * D : b.obs + (e0 * A + lane) * D;
        float rowv[REGROW ? D_T : 1];
        if (row_on && !(MARLNAV_ABLATE & 16)) {
            RowOut ro;
            if constexpr (REGROW) {
                bool ok = true;
                ro = observe_row_regs<A_T, O_T, !OBS_ONLY, kGuardedFast>(
                    st + 5 * A * el, ob + 2 * S * el, tg + 2 * el, a, rowv, pr, ok);
                if (__builtin_expect(__ballot(!ok) != 0ull, 0) && !ok)  // IEEE redo, rare
                    ro = observe_row_regs<A_T, O_T, !OBS_ONLY, false>(
                        st + 5 * A * el, ob + 2 * S * el, tg + 2 * el, a, rowv, pr, ok);
            } else
                ro = observe_row<A_T, O_T, !OBS_ONLY>(A, O, st + 5 * A * el, ob + 2 * S * el,
                                                      tg + 2 * el, a, out_row, pr);
            if (!OBS_ONLY) {
                rmiss[lane] = ro.r_miss;
                rhit[lane] = ro.r_hit;
                rfl[lane] = ro.flags;
            }
        }
        wave_sync();
        STAMP(3);

        if (!OBS_ONLY) {
            // ---- per-env reductions, terminal logic, masked re-init
            bool fin = false, tr_l = false, co_l = false, ta_l = false;
            if (env_on) {
                const int64_t e = e0 + lane;
                unsigned any_col = 0u, all_in = 1u;
                for (int i = 0; i < A; ++i) {
                    const unsigned f = rfl[lane * A + i];
                    any_col |= f & 1u;
                    all_in &= (f >> 1) & 1u;
                }
                const float *rr = all_in ? rhit : rmiss;
                const float rsum = torch_row_sum(rr + lane * A, A, [](float r) { return r; });
                out_st(&b.reward[e], rsum / (float)A);                     // torch.mean (:233)

                float step_num = step_num_in + 1.0f;               // :96
                const bool truncated = step_num > pr.trunc_after;  // :97
                const bool term_old = term_in != 0;
                const bool terminated = any_col || term_old;       // :213-214
                out_st(&b.terminates[e], (uint8_t)(!term_old && all_in));  // :218-219
                out_st(&b.terminated[e], (uint8_t)terminated);
                out_st(&b.truncated[e], (uint8_t)truncated);
                fin = truncated || terminated;                     // :102-104
                if (fin) {
                    float *sts = st + 5 * A * lane;
                    float *obe = ob + 2 * S * lane;
                    float *tge = tg + 2 * lane;
                    if (b.fresh_states) {  // fresh = the moved state itself when FROM_MOVED
                        const bool moved = (pr.flags & MARLNAV_FRESH_STATES_FROM_MOVED) != 0;
                        for (int i = 0; i < 5 * A; ++i)
                            sts[i] = blend_in(sts[i], moved ? sts[i] : b.fresh_states[e * A * 5 + i]);
                        for (int i = 0; i < 2 * S; ++i)
                            obe[i] = blend_in(obe[i], b.fresh_obstacles[e * S * 2 + i]);
                        tge[0] = blend_in(tge[0], b.fresh_target[2 * e]);
                        tge[1] = blend_in(tge[1], b.fresh_target[2 * e + 1]);
                    } else {
                        native_fresh_env<NOISY>(A, S, pr, b.formation,
                                                (uint64_t)(args.env_offset + e), args.step_idx,
                                                sts, obe, tge);
                    }
                    for (int i = 0; i < 2 * S; ++i) b.obstacles[e * S * 2 + i] = obe[i];
                    b.target[2 * e] = tge[0];
                    b.target[2 * e + 1] = tge[1];
                    step_num = blend_in(step_num, 0.0f);
                }
                out_st(&b.step_num[e], step_num);
                envbits[lane] = fin ? 1u : 0u;
                tr_l = truncated;
                co_l = any_col;
                ta_l = all_in;
            }
            c_trunc += __popcll(__ballot(tr_l));
            c_col += __popcll(__ballot(co_l));
            c_tar += __popcll(__ballot(ta_l));
            const bool any_fin = __ballot(fin) != 0ull;
            wave_sync();
            STAMP(4);

            // ---- observations of re-initialised envs (:105)
            if (any_fin) {
                if (row_on && envbits[el]) {
                    if constexpr (REGROW) {
                        bool ok = true;
                        observe_row_regs<A_T, O_T, false, kGuardedFast>(st + 5 * A * el, ob + 2 * S * el,
                                                                tg + 2 * el, a, rowv, pr, ok);
                        if (!ok)
                            observe_row_regs<A_T, O_T, false, false>(
                                st + 5 * A * el, ob + 2 * S * el, tg + 2 * el, a, rowv, pr, ok);
                    } else
                        observe_row<A_T, O_T, false>(A, O, st + 5 * A * el, ob + 2 * S * el,
                                                     tg + 2 * el, a, out_row, pr);
                }
                wave_sync();
            }
            STAMP(5);
        }

        // ---- stream the tile out
        if constexpr (REGROW) {
            if (row_on) {
                store_row<D_T>(b.obs + (e0 * A + lane) * D_T, rowv);
                if (norm) {
                    float nv[D_T];
#pragma unroll
                    for (int k = 0; k < D_T; ++k)
                        nv[k] = (rowv[k] - b.norm_mean[k]) / b.norm_scale[k];
                    store_row<D_T>(b.obs_norm + (e0 * A + lane) * D_T, nv);
                }
            }
        } else if (wp.obs_lds)
            wave_store(b.obs + e0 * A * D, obs_t, nr * D, lane,
                       norm ? b.obs_norm + e0 * A * D : nullptr, b.norm_mean, b.norm_scale, D);
        else if (norm && row_on)
            for (int k = 0; k < D; ++k)
                b.obs_norm[(e0 * A + lane) * D + k] =
                    (out_row[k] - b.norm_mean[k]) / b.norm_scale[k];
        if (!OBS_ONLY)
            wave_store(b.states + e0 * A * 5, st, nr * 5, lane, nullptr, nullptr, nullptr, 1);
        STAMP(6);
    }
    if (!OBS_ONLY && b.counters && lane == 0) {
        // this wave's own slots: contention-free, fire-and-forget
        if (c_trunc) atomicAdd(&b.counters[0 * args.waves + gw], (unsigned long long)c_trunc);
        if (c_col) atomicAdd(&b.counters[1 * args.waves + gw], (unsigned long long)c_col);
        if (c_tar) atomicAdd(&b.counters[2 * args.waves + gw], (unsigned long long)c_tar);
    }
#if MARLNAV_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(7);
    if (lane == 0) {
        g_stamps[(size_t)gw * 24 + 16] = t_entry;
        g_stamps[(size_t)gw * 24 + 17] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        g_stamps[(size_t)gw * 24 + 18] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
    }
#endif
}

// ------------------------------------------------------- tile step kernel
// The step for compile-time shapes on full, 16-byte aligned tiles (the
// common case: every tile but a partial last one). Same tile/lane mapping
// and phases as wave_kernel, with
//  * staging by LDS-DMA (global_load_lds): each span of the tile is copied
//    global -> LDS by 1-2 wave instructions, no VGPR round trip, all in
//    flight before one vmcnt wait;
//  * the own agent row kept in registers from the move to the observation;
//  * per-agent reward terms packed into one 16-byte LDS slot per row;
//  * kernel arguments that only rare paths use (re-init sources, fused
//    normaliser, counters) read through a late kernarg pointer, so the hot
//    path's scalar registers are not spent holding them.
typedef __attribute__((address_space(3))) void LdsVoid;

struct KArgs {
    StepArgs a;
    MarlnavParams p;
};
typedef __attribute__((address_space(4))) const KArgs KArgsK;

// Kernarg pointer the compiler cannot hoist loads through.
__device__ __forceinline__ KArgsK *kargs_late()
{
    KArgsK *k = (KArgsK *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k));
    return k;
}

template <class T>
__device__ __forceinline__ T in_sgpr(T p)
{
    asm volatile("" : "+s"(p));
    return p;
}

// Per-tile snapshot of the hot-path pointers and parameters, read through a
// fresh opaque kernarg pointer each tile: nothing derived from them is
// loop-invariant to the compiler, so a multi-tile loop keeps no per-pointer
// induction variables or hoisted copies alive across tiles.
struct StepPtrs {
    float *states, *obstacles, *target, *step_num, *obs, *reward;
    uint8_t *terminates, *terminated, *truncated;
    const float *actions, *formation;
};

__device__ __forceinline__ StepPtrs load_ptrs(KArgsK *K)
{
    StepPtrs q;
    q.states = K->a.b.states;
    q.obstacles = K->a.b.obstacles;
    q.target = K->a.b.target;
    q.step_num = K->a.b.step_num;
    q.obs = K->a.b.obs;
    q.reward = K->a.b.reward;
    q.terminates = K->a.b.terminates;
    q.terminated = K->a.b.terminated;
    q.truncated = K->a.b.truncated;
    q.actions = K->a.b.actions;
    q.formation = K->a.b.formation;
    return q;
}

__device__ __forceinline__ MarlnavParams load_params(KArgsK *K)
{
    MarlnavParams p;
#define MARLNAV_CP(f) p.f = K->p.f
    MARLNAV_CP(min_speed); MARLNAV_CP(max_speed); MARLNAV_CP(min_accel); MARLNAV_CP(max_accel);
    MARLNAV_CP(trunc_after); MARLNAV_CP(risk_factor); MARLNAV_CP(distance_factor);
    MARLNAV_CP(heading_factor); MARLNAV_CP(target_factor); MARLNAV_CP(soft_factor);
    MARLNAV_CP(bond_factor); MARLNAV_CP(ob_risk_dist); MARLNAV_CP(ag_risk_dist);
    MARLNAV_CP(ob_coll_dist); MARLNAV_CP(ag_coll_dist); MARLNAV_CP(agents_min_d);
    MARLNAV_CP(agents_max_d); MARLNAV_CP(max_at_prop_d); MARLNAV_CP(max_angle_diff);
    MARLNAV_CP(target_radius); MARLNAV_CP(cap_distance); MARLNAV_CP(bond_sharpness);
    MARLNAV_CP(ideal_dist); MARLNAV_CP(init_dist); MARLNAV_CP(obs_range_x);
    MARLNAV_CP(obs_mean_x); MARLNAV_CP(obs_range_y); MARLNAV_CP(obs_mean_y);
    MARLNAV_CP(ags_dist); MARLNAV_CP(noise_std); MARLNAV_CP(angle_range);
    MARLNAV_CP(flags); MARLNAV_CP(seed);
    MARLNAV_CP(act_scale[0]); MARLNAV_CP(act_scale[1]);
    MARLNAV_CP(act_mean[0]); MARLNAV_CP(act_mean[1]);
#undef MARLNAV_CP
    p.reserved = 0;
    return p;
}

// global -> LDS copy of NB bytes (multiple of 4) by LDS-DMA: 16 bytes per lane
// per instruction, then single dwords. src (16-byte aligned) and dst are
// wave-uniform.
template <int NB>
#ifndef MARLNAV_GLDS_AUX  // cache-policy bits of the LDS-DMA staging loads (timing builds)
#define MARLNAV_GLDS_AUX 0
#endif
__device__ __forceinline__ void glds_span(const void *src, float *dst, unsigned lane)
{
    constexpr int N16 = NB / 16, R4 = (NB % 16) / 4;
#pragma unroll
    for (int k = 0; k * 64 < N16; ++k) {
        const char *s = in_sgpr(reinterpret_cast<const char *>(src) + k * 1024);
        if ((k + 1) * 64 <= N16 || (int)lane < N16 - k * 64)
            __builtin_amdgcn_global_load_lds(s + lane * 16u, (LdsVoid *)(dst + k * 256), 16, 0,
                                             MARLNAV_GLDS_AUX);
    }
    if constexpr (R4 > 0) {
        const char *s = in_sgpr(reinterpret_cast<const char *>(src) + N16 * 16);
        if ((int)lane < R4)
            __builtin_amdgcn_global_load_lds(s + lane * 4u, (LdsVoid *)(dst + N16 * 4), 4, 0,
                                             MARLNAV_GLDS_AUX);
    }
}

// plain copy of n elements (partial tiles)
template <class T>
__device__ __forceinline__ void copy_span(const T *__restrict__ src, T *__restrict__ dst, int n,
                                          int lane)
{
#pragma clang loop vectorize(disable) unroll(disable)
    for (int i = lane; i < n; i += 64) dst[i] = src[i];
}

__host__ __device__ constexpr int tile_envs(int A) { return (64 / A) >= 4 ? (64 / A) & ~3 : 64 / A; }


// ------------------------------------------------------ pair-split kernel
// For shapes whose rows carry many pairs (A16/O32: 48 per row) or grids too
// small to fill the chip with one lane per row: LPR lanes share each agent
// row. Lane q of a row evaluates the target pair (kept by q == 0), obstacles
// q, q+LPR, ... and other agents q, q+LPR, ...; the packed observation rows
// are assembled in LDS and streamed out with vector stores; per-row flags
// and counts are OR/sum-reduced across the LPR lanes with DPP / swizzles;
// the row's bond terms (environment.py:264-269) are evaluated by the lanes
// that own the distances and summed by the row leader in torch's order.
// LDS row stride of the split kernel's packed observation rows: D padded
// (keeping 16-byte row alignment when D % 4 == 0) so that the LPR lanes of
// each of the 32/LPR rows in a ds_write_b32 lane group hit distinct banks
// ((a/4) mod 32, MI355X_MICROARCH.md §LDS). At A16/O32 (D = 96) unpadded rows
// are 8-way conflicted: every row starts on bank 0.
__host__ __device__ constexpr int split_conflicts(int s, int LPR, int rows)
{
    int worst = 0;
    for (int b = 0; b < 32; ++b) {
        int n = 0;
        for (int l = 0; l < 32; ++l) {
            const int r = l / LPR, q = l % LPR;
            if (r < rows && (r * s + q) % 32 == b) ++n;
        }
        worst = n > worst ? n : worst;
    }
    return worst;
}

__host__ __device__ constexpr int split_row_stride(int D, int LPR, int rows)
{
    if (D % 4 != 0) return D;  // rows stored with 4/8-byte pieces: keep them dense
    int best = D, bc = split_conflicts(D, LPR, rows);
    for (int s = D + 4; s <= D + 32; s += 4) {
        const int c = split_conflicts(s, LPR, rows);
        if (c < bc) {
            best = s;
            bc = c;
        }
    }
    return best;
}

// ------------------------------------- workgroup-spread re-init / re-observe
// Where the block-spread re-init / re-observation below finds an env of the
// workgroup: `c` is an env code from the finished-env list. BlockEnvs: the
// env-block kernel's block-wide arrays (code = env within the block);
// SplitEnvs: the pair-split kernel's wave-private tiles (code = wave * EPW +
// env within the wave's tile, the tiles of a workgroup being consecutive).
template <int A, int O, int RS>
struct BlockEnvs {
    float *st, *ob, *tg, *rows;
    int64_t e0;
    __device__ float *state(int c) const { return st + 5 * A * c; }
    __device__ float *obst(int c) const { return ob + 2 * O * c; }
    __device__ float *targ(int c) const { return tg + 2 * c; }
    __device__ float *row(int c, int ag) const { return rows + (c * A + ag) * RS; }
    __device__ int64_t env(int c) const { return e0 + c; }
};

template <int A, int O, int EPW, int FLOATS, int ST, int OB, int TG, int OBS, int RS>
struct SplitEnvs {
    float *lds;
    int64_t e0;
    __device__ float *wave(int c) const { return lds + (c / EPW) * FLOATS; }
    __device__ float *state(int c) const { return wave(c) + ST + 5 * A * (c % EPW); }
    __device__ float *obst(int c) const { return wave(c) + OB + 2 * O * (c % EPW); }
    __device__ float *targ(int c) const { return wave(c) + TG + 2 * (c % EPW); }
    __device__ float *row(int c, int ag) const { return wave(c) + OBS + ((c % EPW) * A + ag) * RS; }
    __device__ int64_t env(int c) const { return e0 + c; }
};

// Re-observation of the finished envs (environment.py:105) spread over the
// workgroup: one (row, pair) item per thread per pass, results written
// straight into the packed rows. Per wave and pass, the short sqrt/division
// sequences run when every coordinate of the pass passes coord_ok, IEEE
// otherwise.
template <int A, int O, class Envs, class List>
__device__ __forceinline__ void reobs_block(const Envs &ev, const List &list, int nfin, float cap,
                                            int tid, int nt)
{
    constexpr int NP = 1 + O + (A - 1);
    const int nw = nfin * A * NP;
    for (int base = 0; base < nw; base += nt) {
        const int w = base + tid;
        const bool on = w < nw;
        const int wc = on ? w : 0;
        const int fe = wc / (A * NP), rem = wc - fe * (A * NP);
        const int ag = rem / NP, p = rem - ag * NP;
        const int c = list[fe];
        const float *s = ev.state(c) + 5 * ag;
        const float ox = s[0], oy = s[1], dx = s[2], dy = s[3];
        const float *pt;
        int sa, sd;
        if (p == 0) {            // target
            pt = ev.targ(c);
            sa = 0;
            sd = 1;
        } else if (p <= O) {     // obstacle p - 1
            pt = ev.obst(c) + 2 * (p - 1);
            sa = 1 + p;
            sd = 1 + O + p;
        } else {                 // other agent kx, skipping self
            const int kx = p - O - 1;
            pt = ev.state(c) + 5 * (kx + (kx >= ag ? 1 : 0));
            sa = 2 + 2 * O + kx;
            sd = 2 + 2 * O + (A - 1) + kx;
        }
        const float px = pt[0], py = pt[1];
        const bool cok = coord_ok(ox) && coord_ok(oy) && coord_ok(px) && coord_ok(py);
        bool unused = true;
        float d, ang;
        if (__ballot(on && !cok) == 0ull) {
            d = pair_dist<true>(ox, oy, px, py, unused);
            ang = pair_angle<true>(ox, oy, px, py, dx, dy, d, cap, unused);
        } else {
            d = pair_dist<false>(ox, oy, px, py, unused);
            ang = pair_angle<false>(ox, oy, px, py, dx, dy, d, cap, unused);
        }
        if (on) {
            float *o = ev.row(c, ag);
            o[sa] = ang;
            o[sd] = d;
        }
    }
}

template <int D>
__device__ __forceinline__ void lds_row_write(float *dst, const float *row)
{
    if constexpr (D % 4 == 0) {
#pragma unroll
        for (int k = 0; k < D; k += 4)
            *reinterpret_cast<float4 *>(dst + k) = make_float4(row[k], row[k + 1], row[k + 2], row[k + 3]);
    } else if constexpr (D % 2 == 0) {
#pragma unroll
        for (int k = 0; k < D; k += 2)
            *reinterpret_cast<float2 *>(dst + k) = make_float2(row[k], row[k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < D; ++k) dst[k] = row[k];
    }
}

// Re-initialisation of the finished envs (environment.py:76-90, the sampler
// call at :78) spread over the workgroup: one item per thread per pass - one
// float of a fresh candidate (reference RNG) or of the formation template,
// or one Philox block of two obstacles (native; the same draws as
// native_fresh_env). Writes the LDS state and the global obstacles / target;
// the agent rows go out with the final stores.
template <int A, int O, class Envs, class List>
__device__ __forceinline__ void reinit_block(KArgsK *kl, const Envs &ev, const float *form,
                                             const List &list, int nfin, int tid, int nt)
{
    float *gob = kl->a.b.obstacles;
    float *gtg = kl->a.b.target;
    const float *fs = kl->a.b.fresh_states;
    if (fs) {
        const float *fo = kl->a.b.fresh_obstacles, *ft = kl->a.b.fresh_target;
        const bool keep = (kl->p.flags & MARLNAV_FRESH_STATES_FROM_MOVED) != 0;
        constexpr int NI = 5 * A + 2 * O + 2;
        for (int i = tid; i < nfin * NI; i += nt) {
            const int fe = i / NI, kk = i - fe * NI;
            const int c = list[fe];
            const int64_t e = ev.env(c);
            if (kk < 5 * A) {
                float *d = ev.state(c) + kk;
                *d = blend_in(*d, keep ? *d : fs[e * A * 5 + kk]);
            } else if (kk < 5 * A + 2 * O) {
                const int j = kk - 5 * A;
                float *d = ev.obst(c) + j;
                const float v = blend_in(*d, fo[e * O * 2 + j]);
                *d = v;
                gob[e * O * 2 + j] = v;
            } else {
                const int j = kk - 5 * A - 2 * O;
                float *d = ev.targ(c) + j;
                const float v = blend_in(*d, ft[2 * e + j]);
                *d = v;
                gtg[2 * e + j] = v;
            }
        }
        return;
    }
    constexpr int NB = (O + 1) / 2, NI = 5 * A + 2 + NB;
    const uint64_t seed = kl->p.seed, sidx = kl->a.step_idx;
    const int64_t eoff = kl->a.env_offset;
    const float rx = kl->p.obs_range_x, mx = kl->p.obs_mean_x;
    const float ry = kl->p.obs_range_y, my = kl->p.obs_mean_y;
    for (int i = tid; i < nfin * NI; i += nt) {
        const int fe = i / NI, kk = i - fe * NI;
        const int c = list[fe];
        const int64_t e = ev.env(c);
        if (kk < 5 * A) {
            float *d = ev.state(c) + kk;
            *d = blend_in(*d, form[kk]);
        } else if (kk < 5 * A + 2) {
            const int j = kk - 5 * A;
            float *d = ev.targ(c) + j;
            const float v = blend_in(*d, form[kk]);
            *d = v;
            gtg[2 * e + j] = v;
        } else {
            const int jb = kk - 5 * A - 2;  // obstacles 2jb, 2jb + 1
            const uint64_t gid = (uint64_t)(eoff + e);
            uint32_t cc[4] = {(uint32_t)jb, (uint32_t)sidx, (uint32_t)gid,
                              (uint32_t)(gid >> 32) ^ ((uint32_t)(sidx >> 32) << 16)};
            philox4x32_10(cc, (uint32_t)seed, (uint32_t)(seed >> 32));
            const int j = 2 * jb;
            float *o = ev.obst(c) + 2 * j;
            float *g = gob + e * O * 2 + 2 * j;
            o[0] = g[0] = blend_in(o[0], rx * ((float)(cc[0] >> 8) * 0x1.0p-24f - 0.5f) + mx);
            o[1] = g[1] = blend_in(o[1], ry * ((float)(cc[1] >> 8) * 0x1.0p-24f - 0.5f) + my);
            if (j + 1 < O) {
                o[2] = g[2] = blend_in(o[2], rx * ((float)(cc[2] >> 8) * 0x1.0p-24f - 0.5f) + mx);
                o[3] = g[3] = blend_in(o[3], ry * ((float)(cc[3] >> 8) * 0x1.0p-24f - 0.5f) + my);
            }
        }
    }
}

// Native (non-noisy) re-init and re-observation of the finished envs in ONE
// pass over the workgroup: a fresh env's agent rows and target are the
// formation template and its obstacles are Philox draws (the same as
// native_fresh_env), so each observation item computes its own inputs
// instead of waiting for a re-init pass and a barrier. Items per finished
// env: A*(1+O+A-1) pairs (written into the packed rows), 5A+2 template
// floats and ceil(O/2) Philox blocks (written to the LDS state and the
// global obstacles/target).
template <int A, int O, class Envs, class List>
__device__ __forceinline__ void reinit_reobs_native(KArgsK *kl, const Envs &ev, const float *form,
                                                    const List &list, int nfin, float cap, int tid,
                                                    int nt)
{
    constexpr int NP = 1 + O + (A - 1), NB = (O + 1) / 2;
    constexpr int NPAIR = A * NP, NI = NPAIR + 5 * A + 2 + NB;
    const uint64_t seed = kl->p.seed, sidx = kl->a.step_idx;
    const int64_t eoff = kl->a.env_offset;
    const float rx = kl->p.obs_range_x, mx = kl->p.obs_mean_x;
    const float ry = kl->p.obs_range_y, my = kl->p.obs_mean_y;
    float *gob = kl->a.b.obstacles;
    float *gtg = kl->a.b.target;
    const int n = nfin * NI;
    for (int base = 0; base < n; base += nt) {
        const int i = base + tid;
        const bool on = i < n;
        const int ic = on ? i : 0;
        const int fe = ic / NI, kk = ic - fe * NI;
        const int c = list[fe];
        const int64_t e = ev.env(c);
        const uint64_t gid = (uint64_t)(eoff + e);
        const bool pair = kk < NPAIR;
        // Philox block: obstacle pair items (the block of their obstacle) and
        // obstacle store items
        int jb = -1;
        int ag = 0, p = 0;
        if (pair) {
            ag = kk / NP;
            p = kk - ag * NP;
            if (p >= 1 && p <= O) jb = (p - 1) >> 1;
        } else if (kk >= NPAIR + 5 * A + 2) {
            jb = kk - (NPAIR + 5 * A + 2);
        }
        uint32_t cc[4] = {0u, 0u, 0u, 0u};
        if (jb >= 0) {
            cc[0] = (uint32_t)jb;
            cc[1] = (uint32_t)sidx;
            cc[2] = (uint32_t)gid;
            cc[3] = (uint32_t)(gid >> 32) ^ ((uint32_t)(sidx >> 32) << 16);
            philox4x32_10(cc, (uint32_t)seed, (uint32_t)(seed >> 32));
        }
        if (pair) {
            // inputs: the blend of the env's current value (LDS; other items
            // may be blending it in place meanwhile - blend_in is idempotent)
            // with its fresh value (template or Philox draw)
            const float *s = form + 5 * ag;
            const float *so = ev.state(c) + 5 * ag;
            const float ox = blend_in(so[0], s[0]), oy = blend_in(so[1], s[1]);
            const float dx = blend_in(so[2], s[2]), dy = blend_in(so[3], s[3]);
            float px, py;
            int sa, sd;
            if (p == 0) {            // target
                px = blend_in(ev.targ(c)[0], form[5 * A]);
                py = blend_in(ev.targ(c)[1], form[5 * A + 1]);
                sa = 0;
                sd = 1;
            } else if (p <= O) {     // obstacle p - 1: components of its Philox block
                const bool hi = ((p - 1) & 1) != 0;
                const uint32_t ux = hi ? cc[2] : cc[0], uy = hi ? cc[3] : cc[1];
                const float *oo = ev.obst(c) + 2 * (p - 1);
                px = blend_in(oo[0], rx * ((float)(ux >> 8) * 0x1.0p-24f - 0.5f) + mx);
                py = blend_in(oo[1], ry * ((float)(uy >> 8) * 0x1.0p-24f - 0.5f) + my);
                sa = 1 + p;
                sd = 1 + O + p;
            } else {                 // other agent kx, skipping self
                const int kx = p - O - 1;
                const int m = kx + (kx >= ag ? 1 : 0);
                const float *q = form + 5 * m;
                const float *qo = ev.state(c) + 5 * m;
                px = blend_in(qo[0], q[0]);
                py = blend_in(qo[1], q[1]);
                sa = 2 + 2 * O + kx;
                sd = 2 + 2 * O + (A - 1) + kx;
            }
            const bool cok = coord_ok(ox) && coord_ok(oy) && coord_ok(px) && coord_ok(py);
            bool unused = true;
            float d, ang;
            if (__ballot(on && !cok) == 0ull) {
                d = pair_dist<true>(ox, oy, px, py, unused);
                ang = pair_angle<true>(ox, oy, px, py, dx, dy, d, cap, unused);
            } else {
                d = pair_dist<false>(ox, oy, px, py, unused);
                ang = pair_angle<false>(ox, oy, px, py, dx, dy, d, cap, unused);
            }
            if (on) {
                float *o = ev.row(c, ag);
                o[sa] = ang;
                o[sd] = d;
            }
        } else if (on) {
            const int k2 = kk - NPAIR;
            if (k2 < 5 * A) {
                float *d = ev.state(c) + k2;
                *d = blend_in(*d, form[k2]);
            } else if (k2 < 5 * A + 2) {
                const int j = k2 - 5 * A;
                float *d = ev.targ(c) + j;
                const float v = blend_in(*d, form[k2]);
                *d = v;
                gtg[2 * e + j] = v;
            } else {
                const int j = 2 * jb;
                float *o = ev.obst(c) + 2 * j;
                float *g = gob + e * O * 2 + 2 * j;
                o[0] = g[0] = blend_in(o[0], rx * ((float)(cc[0] >> 8) * 0x1.0p-24f - 0.5f) + mx);
                o[1] = g[1] = blend_in(o[1], ry * ((float)(cc[1] >> 8) * 0x1.0p-24f - 0.5f) + my);
                if (j + 1 < O) {
                    o[2] = g[2] = blend_in(o[2], rx * ((float)(cc[2] >> 8) * 0x1.0p-24f - 0.5f) + mx);
                    o[3] = g[3] = blend_in(o[3], ry * ((float)(cc[3] >> 8) * 0x1.0p-24f - 0.5f) + my);
                }
            }
        }
    }
}

// Finished envs of a split-kernel workgroup: wave w listed cnt[w] env codes
// (w * EPW + env) in slot[w * EPW ...]; entry fe of the concatenation.
template <int EPW>
struct SplitFinList {
    int off1, off2, off3, n;  // prefix sums over the (up to 4) live waves
    const int *slot;
    __device__ static SplitFinList make(const int *cnt, const int *slot, int live)
    {
        static_assert(kWavesPerBlock == 4, "four waves per workgroup");
        const int c0 = cnt[0];
        const int c1 = live > 1 ? cnt[1] : 0;
        const int c2 = live > 2 ? cnt[2] : 0;
        const int c3 = live > 3 ? cnt[3] : 0;
        return SplitFinList{c0, c0 + c1, c0 + c1 + c2, c0 + c1 + c2 + c3, slot};
    }
    __device__ int total() const { return n; }
    __device__ int operator[](int fe) const
    {
        const int w = (fe >= off1) + (fe >= off2) + (fe >= off3);
        const int base = w == 0 ? 0 : (w == 1 ? off1 : (w == 2 ? off2 : off3));
        return slot[w * EPW + fe - base];
    }
};

// Finished envs re-initialised and re-observed by the whole workgroup
// (after one block barrier) instead of by their own wave: pays where an
// env's re-observation is long (measured: A3/O8 and A16/O32 faster, A3/O3
// slower). MARLNAV_SPLIT_SPREAD=0 turns it off (A/B builds).
#ifndef MARLNAV_SPLIT_SPREAD
#define MARLNAV_SPLIT_SPREAD 1
#endif
template <int A, int O>
constexpr bool kSplitSpread = MARLNAV_SPLIT_SPREAD != 0 && A * (1 + O + (A - 1)) >= 32;

template <int A, int O, int LPR>
struct SplitPlan {
    static constexpr int EPW = 64 / LPR / A;  // envs per wave
    static constexpr int R = EPW * A;         // rows per wave
    static constexpr int D = 2 + 2 * O + 2 * (A - 1);
    static constexpr int NOB = (O + LPR - 1) / LPR;        // obstacle pairs per lane
    static constexpr int NAG = (A - 1 + LPR - 1) / LPR;    // other-agent pairs per lane
    static constexpr int ST = 0;                           // (R, 5)
    static constexpr int ACT = (ST + R * 5 + 3) & ~3;      // (R, 2)
    static constexpr int OB = (ACT + R * 2 + 3) & ~3;      // (EPW, O, 2)
    static constexpr int TG = (OB + EPW * O * 2 + 3) & ~3; // (EPW, 2)
    static constexpr int SN = (TG + EPW * 2 + 3) & ~3;     // (EPW,)
    static constexpr int DP = split_row_stride(D, LPR, R < 32 / LPR ? R : 32 / LPR);
    static constexpr int OBS = (SN + EPW + 3) & ~3;        // (R, DP)
    static constexpr int BOND = (OBS + R * DP + 3) & ~3;   // (R, A-1)
    static constexpr int RED = (BOND + R * (A - 1) + 3) & ~3;  // (R, 4)
    static constexpr int FLOATS = RED + 4 * R;
    // after the waves' regions: finished-env counts and slots of the workgroup
    static constexpr int BLK = (kWavesPerBlock * (1 + EPW) + 3) & ~3;
    static_assert(EPW >= 1, "an env's rows must fit one wave");
};

__host__ __device__ constexpr int gcd_c(int a, int b) { return b == 0 ? a : gcd_c(b, a % b); }

// the fast pair math pays for its per-wave coordinate check only with many
// pairs per lane (measured: A16/O32 yes, A3/O3 and A3/O8 at LPR 4 no)
template <int A, int O, int LPR>
constexpr bool kSplitFastMath = SplitPlan<A, O, LPR>::NOB + SplitPlan<A, O, LPR>::NAG >= 6;

// global -> LDS copy of NB bytes whose source is ALIGN-byte aligned: 16-byte
// LDS-DMA when possible, else dword LDS-DMA (NB % 4 == 0, ALIGN % 4 == 0).
template <int NB, int ALIGN>
__device__ __forceinline__ void glds_span_aligned(const void *src, float *dst, unsigned lane)
{
    if constexpr (ALIGN % 16 == 0) {
        glds_span<NB>(src, dst, lane);
    } else {
        static_assert(NB % 4 == 0 && ALIGN % 4 == 0, "dword-aligned span");
        constexpr int N4 = NB / 4;
#pragma unroll
        for (int kk = 0; kk * 64 < N4; ++kk) {
            const char *s = in_sgpr(reinterpret_cast<const char *>(src) + kk * 256);
            if ((kk + 1) * 64 <= N4 || (int)lane < N4 - kk * 64)
                __builtin_amdgcn_global_load_lds(s + lane * 4u, (LdsVoid *)(dst + kk * 64), 4, 0, 0);
        }
    }
}

// OR / sum over the LPR consecutive lanes of a row (LPR a power of two)
template <int LPR>
__device__ __forceinline__ unsigned lpr_or(unsigned v)
{
    if constexpr (LPR >= 2) v |= (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    if constexpr (LPR >= 4) v |= (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    if constexpr (LPR >= 8) v |= (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x101F);
    if constexpr (LPR >= 16) v |= (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x201F);
    return v;
}

template <int LPR>
__device__ __forceinline__ int lpr_sum(int v)
{
    if constexpr (LPR >= 2) v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
    if constexpr (LPR >= 4) v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
    if constexpr (LPR >= 8) v += __builtin_amdgcn_ds_swizzle(v, 0x101F);
    if constexpr (LPR >= 16) v += __builtin_amdgcn_ds_swizzle(v, 0x201F);
    return v;
}

// This lane's pairs of its row: distances and bearings into the LDS row
// `orow`; with TERMS also the per-lane reward flags and bond terms.
struct SplitTerms {
    unsigned fl;  // 1 ob_risk, 2 ob_col, 4 ag_risk, 8 ag_col
    int band;
    float ta, td;
};

// Occupancy the register allocator may assume (waves per SIMD): the grids
// below run at most 3-4 waves per SIMD, so the default target of 8 only
// costs instruction-level parallelism (timing builds set these).
#ifdef MARLNAV_SPLIT_WPE
#define MARLNAV_SPLIT_WPE_ATTR __attribute__((amdgpu_waves_per_eu(MARLNAV_SPLIT_WPE)))
#else
#define MARLNAV_SPLIT_WPE_ATTR
#endif
#ifdef MARLNAV_BLOCK_WPE
#define MARLNAV_BLOCK_WPE_ATTR __attribute__((amdgpu_waves_per_eu(MARLNAV_BLOCK_WPE)))
#else
#define MARLNAV_BLOCK_WPE_ATTR
#endif

// The target pair takes a spare slot of lane LPR-1 when the other agents (or
// else the obstacles) do not divide over the LPR lanes: one pair body fewer per
// wave (A16/O32: 13 -> 12, A3/O8: 4 -> 3); the row leader reads the target
// angle/distance back from the LDS row.
template <int A, int O, int LPR>
constexpr bool kSplitTgtInAg = (A - 1) % LPR != 0;
template <int A, int O, int LPR>
constexpr bool kSplitTgtInOb = !kSplitTgtInAg<A, O, LPR> && O % LPR != 0;

// unroll factor of split_pairs' obstacle / other-agent loops (timing builds)
#ifndef MARLNAV_SPLIT_UNROLL
#define MARLNAV_SPLIT_UNROLL 64
#endif
#define MARLNAV_PRAGMA(x) _Pragma(#x)
#define MARLNAV_UNROLL(n) MARLNAV_PRAGMA(unroll n)

template <int A, int O, int LPR, bool TERMS, bool FAST>
__device__ __forceinline__ SplitTerms split_pairs(const float *__restrict__ sts,
                                                  const float *__restrict__ obe,
                                                  const float *__restrict__ tge, int a, int q,
                                                  float ox, float oy, float dx, float dy,
                                                  float *__restrict__ orow,
                                                  float *__restrict__ bond_row,
                                                  const MarlnavParams &pr, bool &ok)
{
    using SP = SplitPlan<A, O, LPR>;
    constexpr int TQ = LPR - 1;  // the lane whose last other-agent / obstacle slot is spare
    const float cap = pr.cap_distance;
    SplitTerms t{0u, 0, 0.0f, 0.0f};
    if constexpr (!kSplitTgtInAg<A, O, LPR> && !kSplitTgtInOb<A, O, LPR>) {
        const float d = pair_dist<FAST>(ox, oy, tge[0], tge[1], ok);
        const float ang = pair_angle<FAST>(ox, oy, tge[0], tge[1], dx, dy, d, cap, ok);
        t.ta = ang;
        t.td = d;
        if (q == 0) {
            orow[0] = ang;
            orow[1] = d;
        }
    }
    MARLNAV_UNROLL(MARLNAV_SPLIT_UNROLL)
    for (int i = 0; i < SP::NOB; ++i) {
        const int j = q + LPR * i;
        constexpr bool spare = kSplitTgtInOb<A, O, LPR>;
        const bool last = i == SP::NOB - 1;
        const bool valid = O % LPR == 0 || j < O;
        const bool tgt = spare && last && q == TQ;  // j >= O there: the target pair
        if (valid || tgt) {
            const float *pt = tgt ? tge : obe + 2 * (valid ? j : 0);
            const float px = pt[0], py = pt[1];
            const float d = pair_dist<FAST>(ox, oy, px, py, ok);
            const float ang = pair_angle<FAST>(ox, oy, px, py, dx, dy, d, cap, ok);
            if (valid) {
                orow[2 + j] = ang;
                orow[2 + O + j] = d;
                if (TERMS)
                    t.fl |= (d < pr.ob_risk_dist ? 1u : 0u) | (d < pr.ob_coll_dist ? 2u : 0u);
            } else {
                orow[0] = ang;
                orow[1] = d;
            }
        }
    }
    MARLNAV_UNROLL(MARLNAV_SPLIT_UNROLL)
    for (int i = 0; i < SP::NAG; ++i) {
        const int kx = q + LPR * i;  // index among the others
        constexpr bool spare = kSplitTgtInAg<A, O, LPR>;
        const bool last = i == SP::NAG - 1;
        const bool valid = (A - 1) % LPR == 0 || kx < A - 1;
        const bool tgt = spare && last && q == TQ;  // kx >= A - 1 there: the target pair
        if (valid || tgt) {
            const int m = valid ? kx + (kx >= a ? 1 : 0) : 0;
            const float *pt = tgt ? tge : sts + 5 * m;
            const float px = pt[0], py = pt[1];
            const float d = pair_dist<FAST>(ox, oy, px, py, ok);
            const float ang = pair_angle<FAST>(ox, oy, px, py, dx, dy, d, cap, ok);
            if (!valid) {
                orow[0] = ang;
                orow[1] = d;
            } else {
                orow[2 + 2 * O + kx] = ang;
                orow[2 + 2 * O + (A - 1) + kx] = d;
                if (TERMS) {
                    t.fl |= (d < pr.ag_risk_dist ? 4u : 0u) | (d < pr.ag_coll_dist ? 8u : 0u);
                    t.band += (pr.agents_min_d < d && d < pr.agents_max_d) ? 1 : 0;
                    if constexpr (FAST && MARLNAV_FM_TERMS) {
                        const float sd =
                            div_c(d - pr.ideal_dist, make_divc(pr.bond_sharpness, ok), ok);
                        bond_row[kx] = recip_fast(1.0f + sd * sd, ok);
                    } else {
                        const float sd = (d - pr.ideal_dist) / pr.bond_sharpness;
                        bond_row[kx] = 1.0f / (1.0f + sd * sd);
                    }
                }
            }
        }
    }
    return t;
}

template <int A, int O, int LPR, bool OBS_ONLY, bool NOISY>
__global__ void __launch_bounds__(64 * kWavesPerBlock) MARLNAV_SPLIT_WPE_ATTR split_kernel(KArgs k)
{
    using SP = SplitPlan<A, O, LPR>;
    constexpr int EPW = SP::EPW, R = SP::R, D = SP::D;
    (void)k;  // read through kargs_late()
    extern __shared__ __attribute__((aligned(16))) float lds[];
#if MARLNAV_STAMPS
    int stamp_nfin = 0;
#endif
#if MARLNAV_STAMPS
    unsigned long long t_entry;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_entry));
#endif
    const unsigned lane = threadIdx.x & 63;
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t gw = (int64_t)blockIdx.x * kWavesPerBlock + wib;
    const int64_t tile = gw;
    KArgsK *K = kargs_late();
    const int64_t P = K->a.P;
    // pointers first, pinned in SGPRs before the exit test: one round of
    // kernarg loads ahead of the first wait (the compiler would otherwise
    // sink them below the branch, a second serial round)
    const StepPtrs b = load_ptrs(K);
    const int64_t ntiles = K->a.ntiles;
    asm volatile("" ::"s"(b.states), "s"(b.obstacles), "s"(b.target), "s"(b.actions),
                 "s"(b.obs), "s"(ntiles), "s"(P));
    if (tile >= ntiles) return;
    STAMP(0);
    float *wl = lds + wib * SP::FLOATS;
    float *st = wl + SP::ST;
    const int64_t e0 = tile * EPW;
    const int ne = (int)((P - e0) < EPW ? (P - e0) : EPW);
    const int nr = ne * A;

    // ---- stage the tile (the per-env scalars go straight to the env lanes)
    if (ne == EPW) {
        glds_span_aligned<R * 20, gcd_c(R * 20, 16)>(b.states + e0 * (A * 5), st, lane);
        if (!OBS_ONLY)
            glds_span_aligned<R * 8, gcd_c(R * 8, 16)>(b.actions + e0 * (A * 2), wl + SP::ACT, lane);
        glds_span_aligned<EPW * O * 8, gcd_c(EPW * O * 8, 16)>(b.obstacles + e0 * (O * 2),
                                                              wl + SP::OB, lane);
        glds_span_aligned<EPW * 8, gcd_c(EPW * 8, 16)>(b.target + e0 * 2, wl + SP::TG, lane);
    } else {
        copy_span(b.states + e0 * (A * 5), st, nr * 5, (int)lane);
        if (!OBS_ONLY) copy_span(b.actions + e0 * (A * 2), wl + SP::ACT, nr * 2, (int)lane);
        copy_span(b.obstacles + e0 * (O * 2), wl + SP::OB, ne * O * 2, (int)lane);
        copy_span(b.target + e0 * 2, wl + SP::TG, ne * 2, (int)lane);
    }
    const bool env_on = (int)lane < ne;
    float sn_in = 0.0f;
    unsigned term_in = 0u;
    if (!OBS_ONLY && env_on) {
        sn_in = b.step_num[e0 + lane];
        term_in = b.terminates[e0 + lane];
    }
    const MarlnavParams pr = load_params(K);
    const int row = (int)lane / LPR, q = (int)lane - row * LPR;
    const int rowc = row < R ? row : 0;  // idle lanes shadow row 0 (results unused)
    const int el = rowc / A, a = rowc - el * A;
    const bool row_on = row < nr;
    unsigned c_trunc = 0, c_col = 0, c_tar = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS-DMA landed
    wave_sync();
    STAMP(1);

    // ---- _move_agents (environment.py:113-123): every lane of a row moves
    // it (same instructions either way), the row leader stores it
    float ox = st[5 * rowc], oy = st[5 * rowc + 1];
    float dx = st[5 * rowc + 2], dy = st[5 * rowc + 3];
    if (!OBS_ONLY) {
        const float2 act = reinterpret_cast<const float2 *>(wl + SP::ACT)[rowc];
        float a0 = act.x, a1 = act.y;
        if (pr.flags & MARLNAV_SCALE_ACTIONS) {  // ActionScaler (utils.py:546-547)
            KArgsK *kl = kargs_late();
            a0 = kl->p.act_scale[0] * a0 + kl->p.act_mean[0];
            a1 = kl->p.act_scale[1] * a1 + kl->p.act_mean[1];
        }
        float sn, c;
        sincos_k(clamp_t(a0, -kPiF, kPiF), &sn, &c);
        const float ndx = c * dx + (-sn) * dy;
        const float ndy = sn * dx + c * dy;
        const float v = clamp_t(st[5 * rowc + 4] + clamp_t(a1, pr.min_accel, pr.max_accel),
                                pr.min_speed, pr.max_speed);
        ox = ox + ndx * v;
        oy = oy + ndy * v;
        dx = ndx;
        dy = ndy;
        wave_sync();  // every lane has read the pre-move rows
        if (row_on && q == 0) {
            float *s = st + 5 * row;
            s[0] = ox;
            s[1] = oy;
            s[2] = dx;
            s[3] = dy;
            s[4] = v;
        }
        wave_sync();
    }
    STAMP(2);

    // ---- observations + per-lane reward terms (:99-100)
    const float *sts = st + 5 * A * el;
    const float *obe = wl + SP::OB + 2 * O * el;
    const float *tge = wl + SP::TG + 2 * el;
    float *orow = wl + SP::OBS + rowc * SP::DP;
    float *brow = wl + SP::BOND + rowc * (A - 1);
    {
        // wave-uniform choice of the pair math (coord_ok);
        // worth its check only when each lane evaluates many pairs
        bool fast = false;
        if constexpr (kSplitFastMath<A, O, LPR>) {
            const bool cok = (!row_on || (coord_ok(ox) && coord_ok(oy))) &&
                             tile_coords_ok<EPW * O * 2, EPW * 2>(wl + SP::OB, wl + SP::TG, lane);
            fast = ne == EPW && __ballot(!cok) == 0ull;
        }
        bool unused = true;
        SplitTerms t;
        if (__builtin_expect(fast, 1))
            t = split_pairs<A, O, LPR, !OBS_ONLY, true>(sts, obe, tge, a, q, ox, oy, dx, dy, orow,
                                                       brow, pr, unused);
        else
            t = split_pairs<A, O, LPR, !OBS_ONLY, false>(sts, obe, tge, a, q, ox, oy, dx, dy, orow,
                                                        brow, pr, unused);
        if (!OBS_ONLY) {
            const unsigned fl = lpr_or<LPR>(t.fl);
            const int band = lpr_sum<LPR>(t.band);
            wave_sync();  // bond terms of the row are in LDS
            if (row_on && q == 0) {
                if constexpr (kSplitTgtInAg<A, O, LPR> || kSplitTgtInOb<A, O, LPR>) {
                    t.ta = orow[0];  // computed by lane LPR-1 (wave_sync above)
                    t.td = orow[1];
                }
                const float head = fabsf(t.ta) < pr.max_angle_diff ? 1.0f : 0.0f;
                const float bandf = (float)band;
                const float bandc = bandf < pr.max_at_prop_d ? bandf : pr.max_at_prop_d;
                float bv[A - 1];
#pragma unroll
                for (int i = 0; i < A - 1; ++i) bv[i] = brow[i];
                const float bond = torch_row_sum_r<A - 1>(bv, [](float x) { return x; });
                bool okl = MARLNAV_FM_TERMS != 0;
                float dsc = 0.0f, soft = 0.0f, bondm = 0.0f;
                if (MARLNAV_FM_TERMS) {
                    dsc = div_c(bandc, make_divc(pr.max_at_prop_d, okl), okl);
                    soft = -1.0f * div_c(t.td, make_divc(pr.init_dist, okl), okl);
                    bondm = div_c(bond, make_divc((float)(A - 1), okl), okl);
                }
                if (__builtin_expect(!okl, 0)) {
                    dsc = bandc / pr.max_at_prop_d;
                    soft = -1.0f * (t.td / pr.init_dist);
                    bondm = bond / (float)(A - 1);
                }
                const float risk = (fl & 5u) ? 1.0f : 0.0f;
                float rm = pr.target_factor * 0.0f + pr.heading_factor * head;
                float rh = pr.target_factor * 1.0f + pr.heading_factor * head;
                rm = rm + pr.distance_factor * dsc;
                rh = rh + pr.distance_factor * dsc;
                rm = rm + pr.soft_factor * soft;
                rh = rh + pr.soft_factor * soft;
                rm = rm + pr.bond_factor * bondm;
                rh = rh + pr.bond_factor * bondm;
                rm = rm - pr.risk_factor * risk;
                rh = rh - pr.risk_factor * risk;
                const unsigned flags = ((fl & 10u) ? 1u : 0u) | ((t.td < pr.target_radius) ? 2u : 0u);
                reinterpret_cast<float4 *>(wl + SP::RED)[row] =
                    make_float4(rm, rh, __uint_as_float(flags), 0.0f);
            }
        }
    }
    STAMP(3);

    if (!OBS_ONLY) {
        wave_sync();
        // ---- per-env reductions, terminal logic, masked re-init
        bool fin = false, tr_l = false, co_l = false, ta_l = false;
        if (env_on) {
            const int64_t e = e0 + lane;
            const float4 *red = reinterpret_cast<const float4 *>(wl + SP::RED) + A * lane;
            unsigned any_col = 0u, all_in = 1u;
            float rm[A], rh[A];
#pragma unroll
            for (int i = 0; i < A; ++i) {
                const float4 r = red[i];
                const unsigned f = __float_as_uint(r.z);
                any_col |= f & 1u;
                all_in &= (f >> 1) & 1u;
                rm[i] = r.x;
                rh[i] = r.y;
            }
            float rv[A];
#pragma unroll
            for (int i = 0; i < A; ++i) rv[i] = all_in ? rh[i] : rm[i];
            const float rsum = torch_row_sum_r<A>(rv, [](float r) { return r; });
            bool okq = MARLNAV_FM_TERMS != 0;                                    // torch.mean (:233)
            float rmean = MARLNAV_FM_TERMS ? div_c(rsum, make_divc((float)A, okq), okq) : 0.0f;
            if (__builtin_expect(!okq, 0)) rmean = rsum / (float)A;
            out_st(&b.reward[e], rmean);
            float step_num = sn_in + 1.0f;                     // :96
            const bool truncated = step_num > pr.trunc_after;  // :97
            const bool term_old = term_in != 0u;
            const bool terminated = any_col || term_old;       // :213-214
            out_st(&b.terminates[e], (uint8_t)(!term_old && all_in));  // :218-219
            out_st(&b.terminated[e], (uint8_t)terminated);
            out_st(&b.truncated[e], (uint8_t)truncated);
            fin = truncated || terminated;                     // :102-104
            if (fin && (NOISY || !kSplitSpread<A, O>)) {  // per-env re-init on the env lane
                KArgsK *kl = kargs_late();
                MarlnavParams p;  // the fields the re-init reads
                p.obs_range_x = kl->p.obs_range_x;
                p.obs_mean_x = kl->p.obs_mean_x;
                p.obs_range_y = kl->p.obs_range_y;
                p.obs_mean_y = kl->p.obs_mean_y;
                p.ags_dist = kl->p.ags_dist;
                p.noise_std = kl->p.noise_std;
                p.angle_range = kl->p.angle_range;
                p.flags = kl->p.flags;
                p.seed = kl->p.seed;
                float *s5 = st + 5 * A * lane;
                float *obl = wl + SP::OB + 2 * O * lane;
                float *tgl = wl + SP::TG + 2 * lane;
                const float *fs = kl->a.b.fresh_states;
                float *gob = kl->a.b.obstacles;
                float *gtg = kl->a.b.target;
                if (!NOISY && fs) {
                    const float *fo = kl->a.b.fresh_obstacles, *ft = kl->a.b.fresh_target;
                    const bool moved = (p.flags & MARLNAV_FRESH_STATES_FROM_MOVED) != 0;
                    for (int i = 0; i < 5 * A; ++i)
                        s5[i] = blend_in(s5[i], moved ? s5[i] : fs[e * A * 5 + i]);
                    for (int i = 0; i < 2 * O; ++i) obl[i] = blend_in(obl[i], fo[e * O * 2 + i]);
                    tgl[0] = blend_in(tgl[0], ft[2 * e]);
                    tgl[1] = blend_in(tgl[1], ft[2 * e + 1]);
                } else {
                    native_fresh_env<NOISY>(A, O, p, kl->a.b.formation,
                                            (uint64_t)(kl->a.env_offset + e), kl->a.step_idx, s5,
                                            obl, tgl);
                }
                for (int i = 0; i < 2 * O; ++i) gob[e * O * 2 + i] = obl[i];
                gtg[2 * e] = tgl[0];
                gtg[2 * e + 1] = tgl[1];
            }
            if (fin) step_num = blend_in(step_num, 0.0f);
            out_st(&b.step_num[e], step_num);
            tr_l = truncated;
            co_l = any_col;
            ta_l = all_in;
        }
        const uint64_t finmask = __ballot(fin);
        c_trunc = __popcll(__ballot(tr_l));
        c_col = __popcll(__ballot(co_l));
        c_tar = __popcll(__ballot(ta_l));
        STAMP(4);

        if constexpr (kSplitSpread<A, O>) {
            // ---- the workgroup's finished envs, re-initialised (:104) and
            // re-observed (:105) by all its threads: a finished env costs its
            // wave ~1/4 of a full observation pass instead of a second pass
            // on its own lanes (the straggler that set the kernel's end)
            int *bcnt = reinterpret_cast<int *>(lds + kWavesPerBlock * SP::FLOATS);
            int *bslot = bcnt + kWavesPerBlock;
            if (fin)
                bslot[wib * EPW + (int)__builtin_amdgcn_mbcnt_hi(
                                      (unsigned)(finmask >> 32),
                                      __builtin_amdgcn_mbcnt_lo((unsigned)finmask, 0u))] =
                    wib * EPW + (int)lane;
            if (lane == 0) bcnt[wib] = (int)__popcll(finmask);
            __syncthreads();
            const int64_t blk0 = (int64_t)blockIdx.x * kWavesPerBlock;
            const int live = (int)(K->a.ntiles - blk0 < kWavesPerBlock ? K->a.ntiles - blk0
                                                                      : kWavesPerBlock);
            const SplitFinList<EPW> list = SplitFinList<EPW>::make(bcnt, bslot, live);
#if MARLNAV_STAMPS
            stamp_nfin = list.total();
#endif
            if (const int nfin = list.total()) {
                KArgsK *kl = kargs_late();
                const SplitEnvs<A, O, EPW, SP::FLOATS, SP::ST, SP::OB, SP::TG, SP::OBS, SP::DP> ev{
                    lds, blk0 * EPW};
                // waves past the last tile have exited: items go to the live ones
                const int tid = (int)threadIdx.x, nt = 64 * live;
                // fused native re-init + re-observation recomputes a Philox
                // block per obstacle pair: only for few obstacles
                if (!NOISY && O <= 8 && !kl->a.b.fresh_states) {
                    reinit_reobs_native<A, O>(kl, ev, kl->a.b.formation, list, nfin,
                                              pr.cap_distance, tid, nt);
                } else {
                    if (!NOISY) {
                        reinit_block<A, O>(kl, ev, kl->a.b.formation, list, nfin, tid, nt);
                        __syncthreads();
                    }
                    reobs_block<A, O>(ev, list, nfin, pr.cap_distance, tid, nt);
                }
                __syncthreads();
            }
        } else if (finmask) {
            // ---- observations of re-initialised envs (:105), on the wave
            wave_sync();
            const bool redo = row_on && ((finmask >> el) & 1u);
            const float *s = st + 5 * rowc;
            const float rx = s[0], ry = s[1], rdx = s[2], rdy = s[3];
            bool fast2 = false;
            if constexpr (kSplitFastMath<A, O, LPR>) {
                const bool cok2 = (!redo || (coord_ok(rx) && coord_ok(ry))) &&
                                  tile_coords_ok<EPW * O * 2, EPW * 2>(wl + SP::OB, wl + SP::TG, lane);
                fast2 = ne == EPW && __ballot(!cok2) == 0ull;
            }
            bool unused = true;
            if (redo) {
                if (fast2)
                    split_pairs<A, O, LPR, false, true>(sts, obe, tge, a, q, rx, ry, rdx, rdy,
                                                       orow, brow, pr, unused);
                else
                    split_pairs<A, O, LPR, false, false>(sts, obe, tge, a, q, rx, ry, rdx, rdy,
                                                        orow, brow, pr, unused);
            }
        }
    }
    STAMP(5);

    // ---- stream the tile out (obs rows and states from LDS)
    wave_sync();
    {
        const float *src = wl + SP::OBS;
        float *gobs = in_sgpr(b.obs + e0 * (A * D));
        const int n = nr * D;
        constexpr int VAL = gcd_c(R * D * 4, 16);  // tile base alignment in bytes
        float *gnorm = nullptr;
        const float *mean = nullptr, *scale = nullptr;
        if (!OBS_ONLY && (pr.flags & MARLNAV_WRITE_OBS_NORM)) {
            KArgsK *kl = kargs_late();
            gnorm = kl->a.b.obs_norm + e0 * (A * D);
            mean = kl->a.b.norm_mean;
            scale = kl->a.b.norm_scale;
        }
        if constexpr (SP::DP != D) {  // padded rows (D % 4 == 0): 16-byte pieces
            static_assert(D % 4 == 0 && SP::DP % 4 == 0, "padded rows keep 16-byte alignment");
            constexpr int D4 = D / 4;
            if (VAL % 16 == 0) {
                for (int i = (int)lane; i < n / 4; i += 64) {
                    const int rr = i / D4, c4 = i - rr * D4;
                    out_st4<kNtRows>(gobs + 4 * i, *reinterpret_cast<const float4 *>(src + rr * SP::DP + 4 * c4));
                }
            } else {
                for (int i = (int)lane; i < n; i += 64) {
                    const int rr = i / D;
                    out_st<kNtRows>(gobs + i, src[rr * SP::DP + (i - rr * D)]);
                }
            }
        } else if (VAL % 16 == 0 && ne == EPW) {
            for (int i = (int)lane; i < n / 4; i += 64)
                out_st4<kNtRows>(gobs + 4 * i, reinterpret_cast<const float4 *>(src)[i]);
        } else if (VAL % 8 == 0 && n % 2 == 0) {
            for (int i = (int)lane; i < n / 2; i += 64)
                out_st2<kNtRows>(gobs + 2 * i, reinterpret_cast<const float2 *>(src)[i]);
        } else {
            for (int i = (int)lane; i < n; i += 64) out_st<kNtRows>(gobs + i, src[i]);
        }
        if (gnorm)
            for (int i = (int)lane; i < n; i += 64) {
                const int rr = i / D, kk = i - rr * D;
                gnorm[i] = (src[rr * SP::DP + kk] - mean[kk]) / scale[kk];
            }
    }
    if (!OBS_ONLY) {
        float *gst = in_sgpr(b.states + e0 * (A * 5));
        const int n = nr * 5;
        constexpr int SAL = gcd_c(R * 20, 16);
        if (SAL % 16 == 0 && ne == EPW) {
            for (int i = (int)lane; i < n / 4; i += 64)
                out_st4<kNtRows>(gst + 4 * i, reinterpret_cast<const float4 *>(st)[i]);
        } else {
            for (int i = (int)lane; i < n; i += 64) out_st<kNtRows>(gst + i, st[i]);
        }
    }
    STAMP(6);
    if (!OBS_ONLY && lane == 0 && (c_trunc | c_col | c_tar)) {
        KArgsK *kl = kargs_late();
        uint64_t *cnt = kl->a.b.counters;
        const int64_t slots = kl->a.waves;
        if (cnt) {
            const int64_t sl = gw % slots;  // slots may be fewer than this grid's waves
            if (c_trunc) atomicAdd((unsigned long long *)&cnt[0 * slots + sl], (unsigned long long)c_trunc);
            if (c_col) atomicAdd((unsigned long long *)&cnt[1 * slots + sl], (unsigned long long)c_col);
            if (c_tar) atomicAdd((unsigned long long *)&cnt[2 * slots + sl], (unsigned long long)c_tar);
        }
    }
#if MARLNAV_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(7);
    if (lane == 0) {
        g_stamps[(size_t)gw * 24 + 16] = t_entry;
        g_stamps[(size_t)gw * 24 + 17] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        g_stamps[(size_t)gw * 24 + 18] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
        g_stamps[(size_t)gw * 24 + 19] = (unsigned)stamp_nfin;
    }
#endif
}

// ------------------------------------------------------- env-block kernel
// One workgroup of A waves per block of E = 64 consecutive envs: lane l of
// wave w owns agent w of env l. Every lane holds a row (the tile kernels
// leave 64 - 3*20 = 4 lanes idle at A3), the agent index is wave-uniform, and
// the per-env phase runs once per block on wave 0 with all 64 lanes busy
// instead of on 20 of 64 lanes in every wave. Grid shape: at 65536 envs x 3
// agents, 1024 blocks of 3 waves = 3 waves on every SIMD, where 64/3-env
// wave tiles give 3277 waves and a fifth of the SIMDs a fourth wave (measured
// by scripts/kstamps.py: those SIMDs set the kernel's end).
// Rows are exchanged through LDS between block barriers (5 per step); the
// packed observation rows are assembled in LDS and streamed out as one
// contiguous span (a store instruction covers 1 KiB, 8 cache lines, where
// register-row stores at a 48-byte lane stride touch 24).
template <int A, int O>
struct BlockPlan {
    static constexpr int E = 64, R = E * A, D = 2 + 2 * O + 2 * (A - 1);
    static constexpr int NT = 64 * A;                      // threads per block
    static constexpr int ST = 0;                           // (R, 5)
    static constexpr int ACT = (ST + R * 5 + 3) & ~3;      // (R, 2)
    static constexpr int OB = (ACT + R * 2 + 3) & ~3;      // (E, O, 2)
    static constexpr int TG = (OB + E * O * 2 + 3) & ~3;   // (E, 2)
    static constexpr int SN = (TG + E * 2 + 3) & ~3;       // (E,)
    static constexpr int TM = (SN + E + 3) & ~3;           // (E,) bytes
    static constexpr int FORM = (TM + E / 4 + 3) & ~3;     // 5A + 2 (native re-init)
    static constexpr int RED = (FORM + 5 * A + 2 + 3) & ~3;  // (R, 4) reward terms
    static constexpr int OBS = RED + 4 * R;                // (R, D) packed rows
    static constexpr int LIST = (OBS + R * D + 3) & ~3;    // (E,) finished envs
    static constexpr int FLG = LIST + E;                   // [0] nfin, [1 + w] wave w coords bad
    static constexpr int LIST2 = (FLG + 1 + A + 3) & ~3;   // (A-1, E) finished envs, waves >= 1
    static constexpr int FLOATS = (LIST2 + (A - 1) * E + 3) & ~3;
    static_assert(A >= 2 && A <= 16, "one wave per agent");
};

// Copy NB bytes of the block's span k into LDS by LDS-DMA from the wave
// k % A (spans spread over the block's waves).
template <int NB>
__device__ __forceinline__ void block_glds(int k, int A, int w, const void *src, float *dst,
                                           unsigned lane)
{
    if (k % A == w) glds_span<NB>(src, dst, lane);
}

// plain strided copy of n elements by the block's NT threads (partial block)
template <class T>
__device__ __forceinline__ void block_copy(const T *__restrict__ src, T *__restrict__ dst, int n,
                                           int tid, int nt)
{
#pragma clang loop vectorize(disable) unroll(disable)
    for (int i = tid; i < n; i += nt) dst[i] = src[i];
}

// LDS span -> global span of n floats by the block's threads; 16-byte
// vectors for the aligned head (both bases 16-byte aligned by construction)
__device__ __forceinline__ void block_store(float *__restrict__ dst, const float *__restrict__ src,
                                            int n, int tid, int nt)
{
    const int n4 = n >> 2;
    for (int i = tid; i < n4; i += nt)
        out_st4<kNtRows>(dst + 4 * i, reinterpret_cast<const float4 *>(src)[i]);
    for (int i = (n4 << 2) + tid; i < n; i += nt) out_st<kNtRows>(dst + i, src[i]);
}

// block_store of two full spans with compile-time sizes (16-byte aligned,
// multiples of 4 floats): every LDS read of both spans issued before the
// first global store, so the reads' latency is paid once, not per iteration
template <int N1, int N2, int NT>
__device__ __forceinline__ void block_store2(float *__restrict__ d1, const float *__restrict__ s1,
                                             float *__restrict__ d2, const float *__restrict__ s2,
                                             int tid)
{
    static_assert(N1 % 4 == 0 && N2 % 4 == 0, "whole 16-byte pieces");
    constexpr int Q1 = N1 / 4, Q2 = N2 / 4, K1 = (Q1 + NT - 1) / NT, K2 = (Q2 + NT - 1) / NT;
    float4 v1[K1], v2[K2];
#pragma unroll
    for (int k = 0; k < K1; ++k)
        if ((k + 1) * NT <= Q1 || tid + k * NT < Q1)
            v1[k] = reinterpret_cast<const float4 *>(s1)[tid + k * NT];
#pragma unroll
    for (int k = 0; k < K2; ++k)
        if ((k + 1) * NT <= Q2 || tid + k * NT < Q2)
            v2[k] = reinterpret_cast<const float4 *>(s2)[tid + k * NT];
#pragma unroll
    for (int k = 0; k < K1; ++k)
        if ((k + 1) * NT <= Q1 || tid + k * NT < Q1) out_st4<kNtRows>(d1 + 4 * (tid + k * NT), v1[k]);
#pragma unroll
    for (int k = 0; k < K2; ++k)
        if ((k + 1) * NT <= Q2 || tid + k * NT < Q2) out_st4<kNtRows>(d2 + 4 * (tid + k * NT), v2[k]);
}

#ifndef MARLNAV_BLK_EARLY  // 1: stream rows/states out before the per-env phase
#define MARLNAV_BLK_EARLY 0
#endif
#ifndef MARLNAV_BLK_SPREAD  // 1: re-init finished envs spread over the block
#define MARLNAV_BLK_SPREAD 1
#endif
constexpr bool kBlkEarly = MARLNAV_BLK_EARLY != 0;
constexpr bool kBlkSpread = MARLNAV_BLK_SPREAD != 0;
#ifndef MARLNAV_BLK_OVERLAP  // 1: waves 1..A-1 re-init finished envs during the per-env phase
#define MARLNAV_BLK_OVERLAP 1
#endif
constexpr bool kBlkOverlap = MARLNAV_BLK_OVERLAP != 0 && kBlkSpread && !kBlkEarly;
#ifndef MARLNAV_BLK_PRIO  // s_setprio level of blocks with finished envs (0: off)
#define MARLNAV_BLK_PRIO 0
#endif
constexpr int kBlkPrio = MARLNAV_BLK_PRIO;

// Phases (one block barrier after each): stage | move + coordinate check
// (moved states start streaming out) | observe into LDS rows | rows stream
// out while wave 0 runs the per-env phase | re-init, re-observe and re-store
// the finished envs only (none in most blocks).
template <int A, int O, bool OBS_ONLY, bool NOISY>
__global__ void __launch_bounds__(64 * A) MARLNAV_BLOCK_WPE_ATTR block_kernel(KArgs k)
{
    using BP = BlockPlan<A, O>;
    constexpr int E = BP::E, R = BP::R, D = BP::D, NT = BP::NT;
    (void)k;  // read through kargs_late()
    extern __shared__ __attribute__((aligned(16))) float lds[];
#if MARLNAV_STAMPS
    unsigned long long t_entry;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_entry));
#endif
    const int tid = (int)threadIdx.x;
    const unsigned lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // agent of this wave
    const int64_t blk = blockIdx.x;
    const int64_t gw = blk * A + w;  // stamps slot
    KArgsK *K = kargs_late();
    const int64_t P = K->a.P;
    // launch_block's grid is exactly ntiles blocks: no exit test, so the
    // pointer loads below go out in the same round of kernarg loads as P
    const StepPtrs b = load_ptrs(K);
    STAMP(0);
    float *st = lds + BP::ST;
    const int64_t e0 = blk * E;
    const int ne = (int)((P - e0) < E ? (P - e0) : E);
    const bool full = ne == E;

    // ---- stage the block (spans spread over the waves)
    if (full) {
        block_glds<R * 20>(0, A, w, b.states + e0 * (A * 5), st, lane);
        if (!OBS_ONLY) block_glds<R * 8>(1, A, w, b.actions + e0 * (A * 2), lds + BP::ACT, lane);
        block_glds<E * O * 8>(2, A, w, b.obstacles + e0 * (O * 2), lds + BP::OB, lane);
        block_glds<E * 8>(3, A, w, b.target + e0 * 2, lds + BP::TG, lane);
        if (!OBS_ONLY) {
            block_glds<E * 4>(4, A, w, b.step_num + e0, lds + BP::SN, lane);
            block_glds<E>(5, A, w, b.terminates + e0, lds + BP::TM, lane);
            if (b.formation)
                block_glds<(5 * A + 2) * 4>(6, A, w, b.formation, lds + BP::FORM, lane);
        }
    } else {
        const int nr = ne * A;
        block_copy(b.states + e0 * (A * 5), st, nr * 5, tid, NT);
        if (!OBS_ONLY) block_copy(b.actions + e0 * (A * 2), lds + BP::ACT, nr * 2, tid, NT);
        block_copy(b.obstacles + e0 * (O * 2), lds + BP::OB, ne * O * 2, tid, NT);
        block_copy(b.target + e0 * 2, lds + BP::TG, ne * 2, tid, NT);
        if (!OBS_ONLY) {
            block_copy(b.step_num + e0, lds + BP::SN, ne, tid, NT);
            block_copy(b.terminates + e0, reinterpret_cast<uint8_t *>(lds + BP::TM), ne, tid, NT);
            if (b.formation) block_copy(b.formation, lds + BP::FORM, 5 * A + 2, tid, NT);
        }
    }
    const MarlnavParams pr = load_params(K);
    const int l = (int)lane;  // env of this lane within the block
    const int r = l * A + w;  // row of this lane
    const bool row_on = l < ne;
    const int nrow = ne * A;
    int *bad_word = reinterpret_cast<int *>(lds + BP::FLG) + 1;  // any coordinate off the fast range
    if (tid == 0) *bad_word = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA landed
    __syncthreads();
    STAMP(1);

    // obstacle and target coordinates of the block for the pair-math choice
    // (below); read before the move writes LDS, so the reads overlap it
    // (a partial last block takes the IEEE path without checking)
    CoordRange crange;
    if (!(MARLNAV_ABLATE & 128) && full) {
        constexpr int NC = E * O * 2 + E * 2;  // OB and TG are adjacent spans
        static_assert(BP::TG == BP::OB + E * O * 2, "adjacent obstacle/target spans");
#pragma unroll
        for (int k2 = 0; k2 * NT < NC; ++k2) {
            const int i = tid + k2 * NT;
            if ((k2 + 1) * NT <= NC || i < NC) crange.add(lds[BP::OB + i]);
        }
    }

    // ---- _move_agents (environment.py:113-123), own row in registers
    float ox, oy, dx, dy;
    {
        const float *s = st + 5 * r;
        ox = s[0];
        oy = s[1];
        dx = s[2];
        dy = s[3];
    }
    if (!OBS_ONLY) {
        const float2 act = reinterpret_cast<const float2 *>(lds + BP::ACT)[r];
        float a0 = act.x, a1 = act.y;
        if (pr.flags & MARLNAV_SCALE_ACTIONS) {  // ActionScaler (utils.py:546-547)
            KArgsK *kl = kargs_late();
            a0 = kl->p.act_scale[0] * a0 + kl->p.act_mean[0];
            a1 = kl->p.act_scale[1] * a1 + kl->p.act_mean[1];
        }
        float sn, c;
        sincos_k(clamp_t(a0, -kPiF, kPiF), &sn, &c);
        const float ndx = c * dx + (-sn) * dy;
        const float ndy = sn * dx + c * dy;
        float *s = st + 5 * r;
        const float v = clamp_t(s[4] + clamp_t(a1, pr.min_accel, pr.max_accel), pr.min_speed,
                                pr.max_speed);
        ox = ox + ndx * v;
        oy = oy + ndy * v;
        dx = ndx;
        dy = ndy;
        if (row_on) {
            s[0] = ox;
            s[1] = oy;
            s[2] = dx;
            s[3] = dy;
            s[4] = v;
        }
    }
    // block-uniform choice of the pair math: the short sqrt / shared-
    // reciprocal division (equal to IEEE there) when every coordinate of the
    // block (obstacles and targets above, moved agents here) passes coord_ok,
    // IEEE otherwise
    if (!(MARLNAV_ABLATE & 128) && full) {
        crange.add(ox);
        crange.add(oy);
        // one word for the block, written only by waves that found one (all
        // write 1: a benign race); read once after the barrier
        const bool bad = __ballot(!crange.ok()) != 0ull;
        if (lane == 0 && bad) *bad_word = 1;
    }
    __syncthreads();
    STAMP(2);
    // the moved states are final except in finished envs (re-stored below)
    if (kBlkEarly && !OBS_ONLY) block_store(in_sgpr(b.states + e0 * (A * 5)), st, nrow * 5, tid, NT);
    const bool fast = full && ((MARLNAV_ABLATE & 128) || *bad_word == 0);  // 128: timing only

    // ---- observations of the moved state + reward terms (:99-100)
    float4 *red = reinterpret_cast<float4 *>(lds + BP::RED);
    float *obs_rows = lds + BP::OBS;
    if (!(MARLNAV_ABLATE & 16) && row_on) {
        float rowv[D];
        RowOut ro;
        bool unused = true;
        if (__builtin_expect(fast, 1))
            ro = observe_row_own<A, O, !OBS_ONLY, true>(st + 5 * A * l, lds + BP::OB + 2 * O * l,
                                                        lds + BP::TG + 2 * l, w, ox, oy, dx, dy,
                                                        rowv, pr, unused);
        else
            ro = observe_row_own<A, O, !OBS_ONLY, false>(st + 5 * A * l, lds + BP::OB + 2 * O * l,
                                                         lds + BP::TG + 2 * l, w, ox, oy, dx, dy,
                                                         rowv, pr, unused);
        lds_row_write<D>(obs_rows + r * D, rowv);
        if (!OBS_ONLY) red[r] = make_float4(ro.r_miss, ro.r_hit, __uint_as_float(ro.flags), 0.0f);
    }
    __syncthreads();
    STAMP(3);
    // every row streams out now; the finished envs' rows are re-stored below
    float *gobs = in_sgpr(b.obs + e0 * (A * D));
    if (kBlkEarly || OBS_ONLY) block_store(gobs, obs_rows, nrow * D, tid, NT);
    const bool norm = !OBS_ONLY && (pr.flags & MARLNAV_WRITE_OBS_NORM);
    if (norm && kBlkEarly) {
        KArgsK *kl = kargs_late();
        const float *mean = kl->a.b.norm_mean, *scale = kl->a.b.norm_scale;
        float *gn = kl->a.b.obs_norm + e0 * (A * D);
        for (int i = tid; i < nrow * D; i += NT) {
            const int kk = i % D;
            gn[i] = (obs_rows[i] - mean[kk]) / scale[kk];
        }
    }

    if (!OBS_ONLY) {
        int *list = reinterpret_cast<int *>(lds + BP::LIST);
        int *flg = reinterpret_cast<int *>(lds + BP::FLG);
        const BlockEnvs<A, O, D> ev{st, lds + BP::OB, lds + BP::TG, obs_rows, e0};
        // native (non-noisy) re-init: waves 1..A-1 take the finished envs
        // while wave 0 runs the per-env phase (below)
        const bool overlap = !NOISY && kBlkOverlap && !kargs_late()->a.b.fresh_states;
        // ---- per-env reductions, terminal logic (wave 0, one lane per env)
        if (w == 0) {
            const bool env_on = l < ne;
            bool fin = false, tr_l = false, co_l = false, ta_l = false;
            if (env_on) {
                const int64_t e = e0 + l;
                float4 rr[A];
#pragma unroll
                for (int i = 0; i < A; ++i) rr[i] = red[A * l + i];
                unsigned any_col = 0u, all_in = 1u;
#pragma unroll
                for (int i = 0; i < A; ++i) {
                    const unsigned f = __float_as_uint(rr[i].z);
                    any_col |= f & 1u;
                    all_in &= (f >> 1) & 1u;
                }
                float rv[A];
#pragma unroll
                for (int i = 0; i < A; ++i) rv[i] = all_in ? rr[i].y : rr[i].x;
                const float rsum = torch_row_sum_r<A>(rv, [](float x) { return x; });
                out_st(&b.reward[e], rsum / (float)A);                     // torch.mean (:233)

                float step_num = lds[BP::SN + l] + 1.0f;           // :96
                const bool truncated = step_num > pr.trunc_after;  // :97
                const bool term_old = reinterpret_cast<const uint8_t *>(lds + BP::TM)[l] != 0;
                const bool terminated = any_col || term_old;       // :213-214
                out_st(&b.terminates[e], (uint8_t)(!term_old && all_in));  // :218-219
                out_st(&b.terminated[e], (uint8_t)terminated);
                out_st(&b.truncated[e], (uint8_t)truncated);
                fin = truncated || terminated;                     // :102-104
                if (NOISY && fin) {  // noisy native re-init: serial per env
                    KArgsK *kl = kargs_late();
                    {
                        MarlnavParams p;  // the fields the re-init reads
                        p.obs_range_x = kl->p.obs_range_x;
                        p.obs_mean_x = kl->p.obs_mean_x;
                        p.obs_range_y = kl->p.obs_range_y;
                        p.obs_mean_y = kl->p.obs_mean_y;
                        p.ags_dist = kl->p.ags_dist;
                        p.noise_std = kl->p.noise_std;
                        p.angle_range = kl->p.angle_range;
                        p.flags = kl->p.flags;
                        p.seed = kl->p.seed;
                        float *obl = lds + BP::OB + 2 * O * l;
                        float *tgl = lds + BP::TG + 2 * l;
                        native_fresh_env<NOISY>(A, O, p, lds + BP::FORM,
                                                (uint64_t)(kl->a.env_offset + e), kl->a.step_idx,
                                                st + 5 * A * l, obl, tgl);
                        float *gob = kl->a.b.obstacles;
                        for (int i = 0; i < 2 * O; ++i) gob[e * O * 2 + i] = obl[i];
                        kl->a.b.target[2 * e] = tgl[0];
                        kl->a.b.target[2 * e + 1] = tgl[1];
                    }
                }
                out_st(&b.step_num[e], fin ? blend_in(step_num, 0.0f) : step_num);
                tr_l = truncated;
                co_l = any_col;
                ta_l = all_in;
            }
            const uint64_t finmask = __ballot(fin);
            if (kBlkPrio && finmask) __builtin_amdgcn_s_setprio(kBlkPrio);
            if (fin)
                list[__builtin_amdgcn_mbcnt_hi((unsigned)(finmask >> 32),
                                               __builtin_amdgcn_mbcnt_lo((unsigned)finmask, 0u))] = l;
            const unsigned c_trunc = __popcll(__ballot(tr_l));
            const unsigned c_col = __popcll(__ballot(co_l));
            const unsigned c_tar = __popcll(__ballot(ta_l));
            if (lane == 0) {
                flg[0] = (int)__popcll(finmask);
                if (c_trunc | c_col | c_tar) {
                    KArgsK *kl = kargs_late();
                    uint64_t *cnt = kl->a.b.counters;
                    const int64_t slots = kl->a.waves;
                    if (cnt) {
                        const int64_t sl = blk % slots;
                        if (c_trunc) atomicAdd((unsigned long long *)&cnt[0 * slots + sl], (unsigned long long)c_trunc);
                        if (c_col) atomicAdd((unsigned long long *)&cnt[1 * slots + sl], (unsigned long long)c_col);
                        if (c_tar) atomicAdd((unsigned long long *)&cnt[2 * slots + sl], (unsigned long long)c_tar);
                    }
                }
            }
        } else if (overlap) {
            // ---- waves 1..A-1, while wave 0 runs the per-env phase: the
            // finished set from the inputs wave 0 uses (red flags, step_num,
            // terminates), then the native re-init (:104) and re-observation
            // (:105) of those envs. Disjoint LDS: wave 0 reads red/SN/TM; this
            // writes the states, obstacles, target and rows of finished envs.
            bool fin = false;
            if (l < ne) {
                unsigned any_col = 0u;
#pragma unroll
                for (int i = 0; i < A; ++i) any_col |= __float_as_uint(red[A * l + i].z) & 1u;
                fin = lds[BP::SN + l] + 1.0f > pr.trunc_after || any_col != 0u ||
                      reinterpret_cast<const uint8_t *>(lds + BP::TM)[l] != 0;
            }
            const uint64_t fm = __ballot(fin);
            if (fm) {
                // this block now sets the kernel's end: its waves go first on
                // their SIMDs (the other blocks there have slack)
                if (kBlkPrio) __builtin_amdgcn_s_setprio(kBlkPrio);
                int *wlist = reinterpret_cast<int *>(lds + BP::LIST2) + E * (w - 1);
                if (fin)
                    wlist[__builtin_amdgcn_mbcnt_hi(
                        (unsigned)(fm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)fm, 0u))] = l;
                wave_sync();  // every lane of this wave sees its list
                reinit_reobs_native<A, O>(kargs_late(), ev, lds + BP::FORM, wlist,
                                          (int)__popcll(fm), pr.cap_distance, tid - 64, NT - 64);
            }
        }
        __syncthreads();
        STAMP(4);
        const int nfin = flg[0];
        if (nfin && !overlap) {
            // ---- masked re-init (:104) and observations of the re-initialised
            // envs (:105), then their rows and states go out again
            KArgsK *kl = kargs_late();
            if (!NOISY && kBlkSpread && !kl->a.b.fresh_states) {
                reinit_reobs_native<A, O>(kl, ev, lds + BP::FORM, list, nfin, pr.cap_distance,
                                          tid, NT);
            } else {
                if (!NOISY && kBlkSpread) {
                    reinit_block<A, O>(kl, ev, lds + BP::FORM, list, nfin, tid, NT);
                    __syncthreads();
                }
                reobs_block<A, O>(ev, list, nfin, pr.cap_distance, tid, NT);
            }
            __syncthreads();
            constexpr int NI = A * D + 5 * A;
            float *gst = in_sgpr(b.states + e0 * (A * 5));
            for (int i = tid; kBlkEarly && i < nfin * NI; i += NT) {
                const int fe = i / NI, kk = i - fe * NI;
                const int env = list[fe];
                if (kk < A * D) gobs[env * (A * D) + kk] = obs_rows[env * (A * D) + kk];
                else gst[env * (A * 5) + kk - A * D] = st[env * (A * 5) + kk - A * D];
            }
            if (norm && kBlkEarly) {
                KArgsK *kl = kargs_late();
                const float *mean = kl->a.b.norm_mean, *scale = kl->a.b.norm_scale;
                float *gn = kl->a.b.obs_norm + e0 * (A * D);
                for (int i = tid; i < nfin * A * D; i += NT) {
                    const int fe = i / (A * D), kk = i - fe * (A * D);
                    const int o = list[fe] * (A * D) + kk;
                    gn[o] = (obs_rows[o] - mean[kk % D]) / scale[kk % D];
                }
            }
        }
    }
    STAMP(5);
    if (!kBlkEarly && !OBS_ONLY && full && !norm) {  // ---- stream the block out
        block_store2<E * A * D, E * A * 5, NT>(gobs, obs_rows, in_sgpr(b.states + e0 * (A * 5)),
                                               st, tid);  // (E = 64: whole 16-byte pieces)
    } else if (!kBlkEarly && !OBS_ONLY) {
        block_store(gobs, obs_rows, nrow * D, tid, NT);
        if (norm) {
            KArgsK *kl = kargs_late();
            const float *mean = kl->a.b.norm_mean, *scale = kl->a.b.norm_scale;
            float *gn = kl->a.b.obs_norm + e0 * (A * D);
            for (int i = tid; i < nrow * D; i += NT) {
                const int kk = i % D;
                gn[i] = (obs_rows[i] - mean[kk]) / scale[kk];
            }
        }
        block_store(in_sgpr(b.states + e0 * (A * 5)), st, nrow * 5, tid, NT);
    }
    STAMP(6);
#if MARLNAV_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(7);
    if (lane == 0) {
        g_stamps[(size_t)gw * 24 + 16] = t_entry;
        g_stamps[(size_t)gw * 24 + 17] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        g_stamps[(size_t)gw * 24 + 18] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
        g_stamps[(size_t)gw * 24 + 19] = OBS_ONLY ? 0u : (unsigned)reinterpret_cast<const int *>(lds + BP::FLG)[0];
    }
#endif
    (void)gw;
}

// ----------------------------------------------------- native reinit kernel
__global__ void reinit_all_kernel(int64_t P, int A, int S, int64_t env_offset, uint64_t sidx,
                                  MarlnavParams pr, const float *__restrict__ formation,
                                  float *states, float *obstacles, float *target)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P) return;
    if (pr.flags & MARLNAV_NOISY_AGENTS)
        native_fresh_env<true, false>(A, S, pr, formation, (uint64_t)(env_offset + e), sidx,
                               states + e * A * 5, obstacles + e * S * 2, target + 2 * e);
    else
        native_fresh_env<false, false>(A, S, pr, formation, (uint64_t)(env_offset + e), sidx,
                                states + e * A * 5, obstacles + e * S * 2, target + 2 * e);
}

__global__ void counters_total_kernel(const uint64_t *__restrict__ c, int64_t slots,
                                      uint64_t *out3)
{
    // one wave per counter row
    const int row = blockIdx.x;
    const int lane = threadIdx.x;
    unsigned long long acc = 0;
    for (int64_t i = lane; i < slots; i += 64) acc += c[row * slots + i];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if (lane == 0) out3[row] = acc;
}

// ------------------------------------------------------------------ host
struct Launch {
    int W;
    int64_t ntiles, waves, blocks;
    WavePlan plan;
};

// envs per wave tile: 64 / A, rounded down to a multiple of 4 when that
// leaves >= 4 (16-byte aligned tiles), then shrunk to the LDS budget
bool has_variant(int A, int O);

bool rows_in_registers(int A, int O)
{
    return has_variant(A, O) && obs_dim(A, O) <= kRowRegsMaxD;
}

int pick_wave_envs(int A, int O, int S)
{
    int W = 64 / A;
    if (W >= 4) W &= ~3;
    const bool rr = rows_in_registers(A, O);
    while (W > 1 && make_plan(W, A, O, S, rr).floats > kWaveLdsFloats) W >>= 1;
    return W < 1 ? 1 : W;
}

Launch plan_launch(const MarlnavDims *d)
{
    Launch L;
    L.W = pick_wave_envs(d->num_agents, d->num_obstacles, d->obstacle_stride);
    L.plan = make_plan(L.W, d->num_agents, d->num_obstacles, d->obstacle_stride,
                       rows_in_registers(d->num_agents, d->num_obstacles));
    L.ntiles = (d->num_parallel + L.W - 1) / L.W;
    L.waves = (L.ntiles + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock;
    L.blocks = L.waves / kWavesPerBlock;
    return L;
}

int validate(const MarlnavDims *d)
{
    if (!d) return fail(MARLNAV_EINVAL, "dims is NULL");
    if (d->num_parallel < 1)
        return fail(MARLNAV_EINVAL, "num_parallel=%lld < 1", (long long)d->num_parallel);
    if (d->num_agents < 2 || d->num_agents > kMaxAgents)
        return fail(MARLNAV_EINVAL, "num_agents=%d outside [2, %d]", d->num_agents, kMaxAgents);
    if (d->num_obstacles < 1 || d->num_obstacles > d->obstacle_stride)
        return fail(MARLNAV_EINVAL, "num_obstacles=%d outside [1, obstacle_stride=%d]",
                    d->num_obstacles, d->obstacle_stride);
    if (d->obstacle_stride > kMaxStride)
        return fail(MARLNAV_EINVAL, "obstacle_stride=%d > %d", d->obstacle_stride, kMaxStride);
    const Launch L = plan_launch(d);
    if (L.plan.floats > kWaveLdsFloats)
        return fail(MARLNAV_EUNSUPPORTED, "wave tile does not fit LDS for A=%d O=%d S=%d",
                    d->num_agents, d->num_obstacles, d->obstacle_stride);
    return 0;
}

using StepFn = void (*)(StepArgs, MarlnavParams);

struct KernelPair {
    int A, O;
    StepFn step, obs, noisy;
};

const KernelPair kVariants[] = {
    {3, 3, wave_kernel<3, 3, false>, wave_kernel<3, 3, true>, wave_kernel<3, 3, false, true>},
    {3, 8, wave_kernel<3, 8, false>, wave_kernel<3, 8, true>, wave_kernel<3, 8, false, true>},
    {3, 1, wave_kernel<3, 1, false>, wave_kernel<3, 1, true>, wave_kernel<3, 1, false, true>},
    {2, 1, wave_kernel<2, 1, false>, wave_kernel<2, 1, true>, wave_kernel<2, 1, false, true>},
    {16, 32, wave_kernel<16, 32, false>, wave_kernel<16, 32, true>,
     wave_kernel<16, 32, false, true>},
};

// Step kernels that take their arguments through one KArgs block
using TileFn = void (*)(KArgs);

bool aligned(const void *p, uintptr_t n) { return (reinterpret_cast<uintptr_t>(p) & (n - 1)) == 0; }

// pair-split kernels (split_kernel): rows with many pairs, or grids too small
// for one lane per row to fill the chip
struct SplitVariant {
    int A, O, epw;
    TileFn step, obs, noisy;
    size_t lds;
    bool always;  // also for large grids
    int lpr;
};

#define MARLNAV_SPLIT_VARIANT(A, O, LPR, ALWAYS)                                          \
    {A, O, SplitPlan<A, O, LPR>::EPW, split_kernel<A, O, LPR, false, false>,             \
     split_kernel<A, O, LPR, true, false>, split_kernel<A, O, LPR, false, true>,         \
     (size_t)(SplitPlan<A, O, LPR>::FLOATS * kWavesPerBlock + SplitPlan<A, O, LPR>::BLK) * 4, \
     ALWAYS, LPR}
const SplitVariant kSplitVariants[] = {
#ifndef MARLNAV_C4_LPR  // lanes per agent row at A16/O32 (timing builds)
#define MARLNAV_C4_LPR 4
#endif
    MARLNAV_SPLIT_VARIANT(16, 32, MARLNAV_C4_LPR, true),
    MARLNAV_SPLIT_VARIANT(3, 8, 4, false),
    MARLNAV_SPLIT_VARIANT(3, 3, 4, false),
#ifdef MARLNAV_SPLIT33_LPR2
    MARLNAV_SPLIT_VARIANT(3, 3, 2, false),
#endif
    // 8 lanes per row (<= 2 pairs per lane) for grids of at most kSplitTinyWaves
    // LPR=4 waves (measured: 2x3x3 3.89 -> 3.44 us, 1024x3x8 6.31 -> 6.14 us;
    // 2048x3x3 and 4096x3x3 slower)
    MARLNAV_SPLIT_VARIANT(3, 8, 8, false),
    MARLNAV_SPLIT_VARIANT(3, 3, 8, false),
};
constexpr int64_t kSplitTinyWaves = 256;
#undef MARLNAV_SPLIT_VARIANT

// one-lane-per-row grids below kSplitBelowWaves * (pairs per row / 6) waves
// leave most SIMDs idle (measured: 4096x3x3 and 16384x3x8 split faster,
// 16384x3x3 does not)
constexpr int64_t kSplitBelowWaves = 512;

const SplitVariant *select_split(const MarlnavDims *d, const MarlnavStepBuffers &b, bool obs_only,
                                 bool force_size = false)
{
    if (d->obstacle_stride != d->num_obstacles) return nullptr;
    const SplitVariant *v = nullptr;
    for (const SplitVariant &x : kSplitVariants) {
        if (x.A != d->num_agents || x.O != d->num_obstacles) continue;
        if (x.lpr == 8) {  // the tiny-grid form: LPR=4 would leave >3/4 of the SIMDs idle
            const int64_t e4 = 64 / 4 / x.A;
            if ((d->num_parallel + e4 - 1) / e4 > kSplitTinyWaves) continue;
        }
        v = &x;  // the last applicable variant wins
    }
    if (!v) return nullptr;
    const int64_t row_waves = (d->num_parallel + tile_envs(v->A) - 1) / tile_envs(v->A);
    const int64_t pairs = 1 + v->O + (v->A - 1);
    if (!v->always && !force_size && row_waves * 6 >= kSplitBelowWaves * pairs)
        return nullptr;
    if (!aligned(b.states, 16) || !aligned(b.obstacles, 16) || !aligned(b.target, 16) ||
        !aligned(b.obs, 16))
        return nullptr;
    if (!obs_only && !aligned(b.actions, 16)) return nullptr;
    return v;
}

int launch_split(const SplitVariant &v, TileFn fn, const StepArgs &args, const MarlnavParams &pr,
                 void *stream, const char *what)
{
    KArgs ka;
    ka.a = args;
    ka.p = pr;
    ka.a.W = v.epw;
    ka.a.ntiles = (args.P + v.epw - 1) / v.epw;
    const int64_t blocks = (ka.a.ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
    void *kargs[] = {&ka};
    hipError_t e = hipLaunchKernel(reinterpret_cast<const void *>(fn), dim3((unsigned)blocks),
                                   dim3(64 * kWavesPerBlock), kargs, v.lds, (hipStream_t)stream);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return fail(MARLNAV_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
    return 0;
}

// env-block kernels (block_kernel) for these shapes; MARLNAV_BLOCK=0 turns
// them off (A/B timing against the tile kernels)
struct BlockVariant {
    int A, O;
    TileFn step, obs, noisy;
    size_t lds;
};

#define MARLNAV_BLOCK_VARIANT(A, O)                                                    \
    {A, O, block_kernel<A, O, false, false>, block_kernel<A, O, true, false>,          \
     block_kernel<A, O, false, true>, (size_t)BlockPlan<A, O>::FLOATS * 4}
const BlockVariant kBlockVariants[] = {
    MARLNAV_BLOCK_VARIANT(3, 3),
    MARLNAV_BLOCK_VARIANT(3, 8),
    MARLNAV_BLOCK_VARIANT(3, 1),
    MARLNAV_BLOCK_VARIANT(2, 1),
};
#undef MARLNAV_BLOCK_VARIANT

const BlockVariant *select_block(const MarlnavDims *d, const MarlnavStepBuffers &b, bool obs_only)
{
    if (d->obstacle_stride != d->num_obstacles) return nullptr;
    const BlockVariant *v = nullptr;
    for (const BlockVariant &x : kBlockVariants)
        if (x.A == d->num_agents && x.O == d->num_obstacles) v = &x;
    if (!v) return nullptr;
    if (!aligned(b.states, 16) || !aligned(b.obstacles, 16) || !aligned(b.target, 16) ||
        !aligned(b.obs, 16))
        return nullptr;
    if (!obs_only && (!aligned(b.actions, 16) || !aligned(b.step_num, 16) ||
                      !aligned(b.terminates, 16) || (b.formation && !aligned(b.formation, 16))))
        return nullptr;
    return v;
}

int launch_block(const BlockVariant &v, TileFn fn, const StepArgs &args, const MarlnavParams &pr,
                 void *stream, const char *what)
{
    KArgs ka;
    ka.a = args;
    ka.p = pr;
    ka.a.W = BlockPlan<3, 3>::E;
    ka.a.ntiles = (args.P + ka.a.W - 1) / ka.a.W;
    void *kargs[] = {&ka};
    hipError_t e = hipLaunchKernel(reinterpret_cast<const void *>(fn), dim3((unsigned)ka.a.ntiles),
                                   dim3(64 * v.A), kargs, v.lds, (hipStream_t)stream);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return fail(MARLNAV_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
    return 0;
}

bool has_variant(int A, int O)
{
    for (const KernelPair &k : kVariants)
        if (k.A == A && k.O == O) return true;
    return false;
}

KernelPair select_kernels(int A, int O)
{
    for (const KernelPair &k : kVariants)
        if (k.A == A && k.O == O) return k;
    return KernelPair{0, 0, wave_kernel<0, 0, false>, wave_kernel<0, 0, true>,
                      wave_kernel<0, 0, false, true>};
}

StepArgs make_args(const MarlnavDims *d, const Launch &L)
{
    StepArgs a;
    memset(&a, 0, sizeof(a));
    a.P = d->num_parallel;
    a.env_offset = d->env_offset;
    a.ntiles = L.ntiles;
    a.waves = L.waves;
    a.W = L.W;
    a.A = d->num_agents;
    a.O = d->num_obstacles;
    a.S = d->obstacle_stride;
    return a;
}

int launch(StepFn fn, const Launch &L, StepArgs args, MarlnavParams pr, void *stream,
           const char *what)
{
    void *kargs[] = {&args, &pr};
    const size_t lds = (size_t)L.plan.floats * 4 * kWavesPerBlock;
    hipError_t e = hipLaunchKernel(reinterpret_cast<const void *>(fn), dim3((unsigned)L.blocks),
                                   dim3(64 * kWavesPerBlock), kargs, lds, (hipStream_t)stream);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return fail(MARLNAV_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
    return 0;
}

// marlnav_debug_force_family / marlnav_debug_last_family (testing hooks)
int g_family = MARLNAV_FAMILY_AUTO;
thread_local int g_last_family = MARLNAV_FAMILY_AUTO;

bool family_allowed(int f) { return g_family == MARLNAV_FAMILY_AUTO || g_family == f; }

}  // namespace

extern "C" {

int marlnav_abi_version(void) { return MARLNAV_ABI_VERSION; }

int marlnav_debug_force_family(int family)
{
    const int prev = g_family;
    if (family < MARLNAV_FAMILY_AUTO || family > MARLNAV_FAMILY_WAVE)
        return fail(MARLNAV_EINVAL, "unknown kernel family %d", family);
    g_family = family;
    return prev;
}

int marlnav_debug_last_family(void) { return g_last_family; }

#if MARLNAV_STAMPS
int marlnav_debug_stamps(void *buf)
{
    const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf));
    return e == hipSuccess ? 0 : fail(MARLNAV_ELAUNCH, "stamps: %s", hipGetErrorString(e));
}
#endif

const char *marlnav_last_error(void) { return g_err; }

int64_t marlnav_counter_slots(const MarlnavDims *d)
{
    if (validate(d)) return -1;
    return plan_launch(d).waves;
}

namespace {
// Parameter ranges under which the reward terms' divisions by bond_sharpness,
// init_dist and max_at_prop_d (div_c) and the bond reciprocal (recip_fast)
// are exact for every FAST-range distance: divisors in [2^-20, 2^20] (the
// sharpness in [2^-5, 2^20], so |(d - ideal) / sharpness| <= 2^48 and
// 1 + sd^2 <= 2^96), ideal_dist zero or in [2^-40, 2^40] (so d - ideal is
// zero or >= 2^-66 in magnitude).
bool terms_fast_params(const MarlnavParams &p)
{
    const auto in = [](float c, float lo, float hi) {
        const float a = fabsf(c);
        return a >= lo && a <= hi;
    };
    return in(p.bond_sharpness, 0x1p-5f, 0x1p20f) && in(p.init_dist, 0x1p-20f, 0x1p20f) &&
           in(p.max_at_prop_d, 0x1p-20f, 0x1p20f) &&
           (p.ideal_dist == 0.0f || in(p.ideal_dist, 0x1p-40f, 0x1p40f));
}
}  // namespace

int marlnav_step(const MarlnavDims *d, const MarlnavParams *pr_in, const MarlnavStepBuffers *b,
                 uint64_t step_idx, void *stream)
{
    if (!pr_in) return fail(MARLNAV_EINVAL, "params/buffers is NULL");
    MarlnavParams prm = *pr_in;
    prm.flags &= ~kTermsFastFlag;
    if (terms_fast_params(prm)) prm.flags |= kTermsFastFlag;
    const MarlnavParams *pr = &prm;
    if (int rc = validate(d)) return rc;
    if (!pr || !b) return fail(MARLNAV_EINVAL, "params/buffers is NULL");
    if (!b->states || !b->obstacles || !b->target || !b->step_num || !b->terminates ||
        !b->actions || !b->obs || !b->reward || !b->terminated || !b->truncated)
        return fail(MARLNAV_EINVAL, "a required step buffer is NULL");
    if (!b->fresh_states && !b->formation)
        return fail(MARLNAV_EINVAL, "native re-init needs the formation buffer");
    if (b->fresh_states && (!b->fresh_obstacles || !b->fresh_target))
        return fail(MARLNAV_EINVAL, "fresh_states given without fresh_obstacles/target");
    if ((pr->flags & MARLNAV_WRITE_OBS_NORM) && (!b->obs_norm || !b->norm_mean || !b->norm_scale))
        return fail(MARLNAV_EINVAL, "MARLNAV_WRITE_OBS_NORM needs obs_norm/norm_mean/norm_scale");
    if ((reinterpret_cast<uintptr_t>(b->actions) & 7u) != 0)
        return fail(MARLNAV_EINVAL, "actions must be 8-byte aligned");
    const Launch L = plan_launch(d);
    StepArgs args = make_args(d, L);
    args.b = *b;
    args.step_idx = step_idx;
    const bool noisy = !b->fresh_states && (pr->flags & MARLNAV_NOISY_AGENTS);
    const bool fsplit = g_family == MARLNAV_FAMILY_SPLIT;
    if (family_allowed(MARLNAV_FAMILY_SPLIT))
        if (const SplitVariant *v = select_split(d, *b, false, fsplit)) {
            g_last_family = MARLNAV_FAMILY_SPLIT;
            return launch_split(*v, noisy ? v->noisy : v->step, args, *pr, stream, "marlnav_step");
        }
    if (family_allowed(MARLNAV_FAMILY_BLOCK))
        if (const BlockVariant *v = select_block(d, *b, false)) {
            g_last_family = MARLNAV_FAMILY_BLOCK;
            return launch_block(*v, noisy ? v->noisy : v->step, args, *pr, stream, "marlnav_step");
        }
    const KernelPair k = select_kernels(d->num_agents, d->num_obstacles);
    g_last_family = MARLNAV_FAMILY_WAVE;
    return launch(noisy ? k.noisy : k.step, L, args, *pr, stream, "marlnav_step");
}

int marlnav_observe(const MarlnavDims *d, const MarlnavParams *params, const float *states,
                    const float *obstacles, const float *target, float *obs, void *stream)
{
    if (int rc = validate(d)) return rc;
    if (!states || !obstacles || !target || !obs)
        return fail(MARLNAV_EINVAL, "a required observe buffer is NULL");
    const Launch L = plan_launch(d);
    StepArgs args = make_args(d, L);
    args.b.states = const_cast<float *>(states);
    args.b.obstacles = const_cast<float *>(obstacles);
    args.b.target = const_cast<float *>(target);
    args.b.obs = obs;
    MarlnavParams pr;
    memset(&pr, 0, sizeof(pr));
    // the angle cap (environment.py:172-177) is the only parameter observe reads;
    // NULL params: the reference's default (environment.py:65)
    pr.cap_distance = params ? params->cap_distance : 0.1f;
    const bool fsplit = g_family == MARLNAV_FAMILY_SPLIT;
    if (family_allowed(MARLNAV_FAMILY_SPLIT))
        if (const SplitVariant *v = select_split(d, args.b, true, fsplit)) {
            g_last_family = MARLNAV_FAMILY_SPLIT;
            return launch_split(*v, v->obs, args, pr, stream, "marlnav_observe");
        }
    if (family_allowed(MARLNAV_FAMILY_BLOCK))
        if (const BlockVariant *v = select_block(d, args.b, true)) {
            g_last_family = MARLNAV_FAMILY_BLOCK;
            return launch_block(*v, v->obs, args, pr, stream, "marlnav_observe");
        }
    g_last_family = MARLNAV_FAMILY_WAVE;
    return launch(select_kernels(d->num_agents, d->num_obstacles).obs, L, args, pr, stream,
                  "marlnav_observe");
}

int marlnav_reinit_all(const MarlnavDims *d, const MarlnavParams *pr, const float *formation,
                       float *states, float *obstacles, float *target, uint64_t step_idx,
                       void *stream)
{
    if (int rc = validate(d)) return rc;
    if (!pr || !formation || !states || !obstacles || !target)
        return fail(MARLNAV_EINVAL, "a required reinit buffer is NULL");
    const unsigned blocks = (unsigned)((d->num_parallel + 255) / 256);
    hipLaunchKernelGGL(reinit_all_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       d->num_parallel, d->num_agents, d->obstacle_stride, d->env_offset,
                       step_idx, *pr, formation, states, obstacles, target);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(MARLNAV_ELAUNCH, "marlnav_reinit_all: %s", hipGetErrorString(e));
    return 0;
}

int marlnav_counters_total(const MarlnavDims *d, const uint64_t *counters, uint64_t *out3,
                           void *stream)
{
    const int64_t slots = marlnav_counter_slots(d);
    if (slots < 0) return MARLNAV_EINVAL;
    if (!counters || !out3) return fail(MARLNAV_EINVAL, "counters/out3 is NULL");
    hipLaunchKernelGGL(counters_total_kernel, dim3(3), dim3(64), 0, (hipStream_t)stream,
                       counters, slots, out3);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(MARLNAV_ELAUNCH, "marlnav_counters_total: %s", hipGetErrorString(e));
    return 0;
}

}  // extern "C"
