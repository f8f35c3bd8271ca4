// device_math.h - device arithmetic of the step: exact fp32 pair math (cdist / normalize / acos as the reference evaluates them), heading sin/cos, Philox re-init draws, torch-order row sums, the per-row observation, LDS plans.
// Part of libmarlnav.so: included once, by marlnav_step.hip (one translation
// unit), inside its anonymous namespace.
#pragma once

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
// and stay plain, as do the wave kernel's stores.
constexpr bool kNtRows = true;    // rows and states of the block/split kernels
constexpr bool kNtOther = false;  // per-env scalars and the wave kernel
typedef float v4f_t __attribute__((ext_vector_type(4)));
typedef float v2f_t __attribute__((ext_vector_type(2)));

// Every output pointer is a device (global) allocation: cast it to address
// space 1 so the stores are `global_store_*`, not `flat_store_*`. A FLAT
// store counts on LGKM_CNT as well as VM_CNT, so the `s_waitcnt lgkmcnt(0)`
// that a block barrier needs for the wave's LDS writes would also wait for
// the store to leave; a global store counts on VM_CNT only.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T *gptr(T *p)
{
    return (__attribute__((address_space(1))) T *)p;
}

template <bool NT = kNtOther, class T>
__device__ __forceinline__ void out_st(T *p, T v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, gptr(p));
    else
        *gptr(p) = v;
}

template <bool NT = kNtOther>
__device__ __forceinline__ void out_st4(float *p, float4 v)
{
    auto *q = gptr(reinterpret_cast<v4f_t *>(p));
    if constexpr (NT)
        __builtin_nontemporal_store(v4f_t{v.x, v.y, v.z, v.w}, q);
    else
        *q = v4f_t{v.x, v.y, v.z, v.w};
}

// ---------------------------------------------------- written-through outputs
// The env-block kernel's outputs (observation rows, states, per-env scalars)
// leave through buffer stores with a system-scope cache policy (sc0 sc1):
// they are written through the XCD's L2 to memory as they are issued, so the
// end-of-launch L2 write-back - which a plain or `nt` store leaves with every
// dirty line of the launch (14 MB at 65536x3x3, all written in the last
// microsecond) - has nothing left to flush. Buffer stores carry the policy
// as an operand the compiler tracks (an inline-asm global store would hide
// its vmcnt from the waitcnt insertion), and the resource's byte size bounds
// every store to its span. Only launches that write at least
// kWriteThroughMinBytes take this path: below that the end-of-launch
// write-back is short and waiting for memory acknowledgements at the wave's
// end is not (A/B on two boxes, graph replay, nt -> written through:
// 65536x3x3 (14 MB) 8.38 -> 7.84 and 8.52 -> 8.19 us, 4096x16x32 (27 MB)
// 13.97 -> 13.13 and 13.89 -> 13.68, 512x16x32 (3.3 MB) 9.17 -> 9.66, 8192x3x3
// (1.8 MB) 5.57 -> 5.73, 16384x3x3 (3.5 MB) 5.82 -> 5.62 and 5.78 -> 5.80).
// Round 4, this round's kernels, one box (profiles/r04_ab_wt.txt): threshold
// 8 -> 2 MB: 16384x3x3 5.33 -> 5.17 us, 32768x3x3 6.23 -> 5.91, 512x16x32
// 8.31 -> 8.06, 1024x16x32 8.85 -> 8.38; 8192x3x3 (1.8 MB) stays at 5.05
// below it (5.11 written through); 0 MB would take 2x3x3 3.01 -> 3.11.
// Round 6, final kernels, one box, stream launches / graph replay
// (scripts/diag/launch_modes.py, profiles/r06_ab_wt_min.txt): written through
// at every size against the 2 MB threshold: 8192x3x3 (1.8 MB) 5.08 -> 4.88 /
// 4.57 -> 4.34 us, 4096x3x3 4.92 -> 4.83 / 4.41 -> 4.30, 2048x3x8 5.45 ->
// 5.31 / 5.13 -> 5.02, 1024x3x8 (configs[1]) 4.96 -> 4.90 / 4.65 -> 4.59,
// 512x3x8 4.85 -> 4.80 / 4.59 -> 4.54, 256x3x3 4.47 -> 4.48 / 4.13 -> 4.05,
// but 2x3x3 (configs[0]) 2.85 -> 3.24 / 2.75 -> 2.91: the threshold is 64 KB.
// marlnav_step / marlnav_observe set kWriteThroughFlag in
// MarlnavParams.flags; `wt` in the kernels is that bit.
#ifndef MARLNAV_CPOL
#define MARLNAV_CPOL 17  // SC0 | SC1
#endif
constexpr int kCpolOut = MARLNAV_CPOL < 0 ? 0 : MARLNAV_CPOL;
constexpr bool kWtOut = MARLNAV_CPOL >= 0;
constexpr uint32_t kWriteThroughFlag = 1u << 29;  // internal MarlnavParams.flags bit
#ifndef MARLNAV_WT_MIN_KB
#define MARLNAV_WT_MIN_KB 64
#endif
constexpr int64_t kWriteThroughMinBytes = (int64_t)MARLNAV_WT_MIN_KB << 10;
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v2i_t __attribute__((ext_vector_type(2)));

struct OutBuf {
    __amdgpu_buffer_rsrc_t r;
};

// a wave-uniform output span of `bytes` bytes at `base` (raw buffer: stores
// past `bytes` are dropped)
__device__ __forceinline__ OutBuf out_buf(const void *base, uint32_t bytes)
{
    return OutBuf{__builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes,
                                                     0x00020000)};
}

__device__ __forceinline__ void wt_st(OutBuf b, uint32_t off, float v)
{
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(v), b.r, (int)off, 0, kCpolOut);
}

__device__ __forceinline__ void wt_st(OutBuf b, uint32_t off, uint8_t v)
{
    __builtin_amdgcn_raw_buffer_store_b8((char)v, b.r, (int)off, 0, kCpolOut);
}

__device__ __forceinline__ void wt_st2(OutBuf b, uint32_t off, float2 v)
{
    const v2i_t x{__float_as_int(v.x), __float_as_int(v.y)};
    __builtin_amdgcn_raw_buffer_store_b64(x, b.r, (int)off, 0, kCpolOut);
}

__device__ __forceinline__ void wt_st4(OutBuf b, uint32_t off, float4 v)
{
    const v4i_t x{__float_as_int(v.x), __float_as_int(v.y), __float_as_int(v.z),
                  __float_as_int(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(x, b.r, (int)off, 0, kCpolOut);
}

// Element idx of a global output array that a step writes sparsely or one
// scalar per env (reward, flags, step number, re-initialised obstacles and
// targets): a plain store. Written through, these cost the per-env phase
// 0.4 us (the spread per-env phase 1.12 -> 0.68 us with plain stores;
// 65536x3x3 8.36 -> 7.97 us, 4096x16x32 13.60 -> 13.26, A/B), and their
// 0.7 MB leave little for the end-of-launch write-back.
template <class T>
__device__ __forceinline__ void out_el(T *arr, int64_t idx, T v)
{
    out_st(arr + idx, v);
}

template <bool NT = kNtOther>
__device__ __forceinline__ void out_st2(float *p, float2 v)
{
    auto *q = gptr(reinterpret_cast<v2f_t *>(p));
    if constexpr (NT)
        __builtin_nontemporal_store(v2f_t{v.x, v.y}, q);
    else
        *q = v2f_t{v.x, v.y};
}

// The pair math's FAST mode (the shortened sequences, bit-exact inside their
// guards: scripts/probes/fastmath_probe.hip, sqrt_probe.hip) is entered only
// for a block or tile whose every coordinate passed the coordinate check
// (CoordRange / tile_coords_ok), which implies every per-pair guard, so
// there the guards are dead code. The generic wave kernel, which would have
// to evaluate the guards per pair, was measured slower with them and runs
// IEEE-only (kGuardedFast).
constexpr bool kGuardedFast = false;
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

// Correctly rounded sqrt for x in [2^-96, 2^96] or x == 0, in six VALU: the
// reciprocal square root estimate y, s = x*y, one Newton correction
// s + (x - s*s) * y/2 (the residual exact by FMA), then max(., 0), which maps
// x == 0 (0 * inf = NaN) to +0 and is one v_max on an FMA result. Equal to
// the IEEE sqrtf (hipcc's v_sqrt + two-neighbour residual fix-up, nine VALU)
// on every float of the range and zero: checked exhaustively on the GPU
// (scripts/probes/sqrt_rsq_probe.hip, profiles/r03_sqrt_rsq_probe.txt).
// `ok` is cleared outside the range (the caller redoes the row with IEEE
// sqrt).
__device__ __forceinline__ float sqrt_fast(float x, bool &ok)
{
    ok &= (x >= 0x1p-96f && x <= 0x1p96f) || x == 0.0f;
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y, h = 0.5f * y;
    const float e = __builtin_fmaf(-s, s, x);
    return __builtin_fmaxf(__builtin_fmaf(e, h, s), 0.0f);
}

// torch.cdist direct path (environment.py:271-274)
template <bool FAST = false>
__device__ __forceinline__ float pair_dist(float ox, float oy, float px, float py, bool &ok)
{
    const float dx = px - ox, dy = py - oy;
    if (FAST && (MARLNAV_AB & 64)) return dx + dy;  // timing only: trivial pair math
    if constexpr (FAST)
        return sqrt_fast(__builtin_fmaf(dy, dy, dx * dx), ok);
    else
        return __builtin_sqrtf(__builtin_fmaf(dy, dy, dx * dx));
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
    const float q = x * d.r;
    return __builtin_fmaf(__builtin_fmaf(-d.c, q, x), d.r, q);
}

// 1 / den for den in [1, 2^96] (the bond term's 1 + sd^2): v_rcp_f32 and one
// Newton step, which is the correctly rounded reciprocal for every fp32
// significand (scripts/probes/div_exhaustive.hip, check R), hence for every
// den of the range.
__device__ __forceinline__ float recip_fast(float den, bool &ok)
{
    ok &= den <= 0x1p96f;
    const float r = __builtin_amdgcn_rcpf(den);
    return __builtin_fmaf(__builtin_fmaf(-den, r, 1.0f), r, r);
}

// Two correctly rounded quotients over one denominator: v_rcp_f32 refined by
// one Newton step (r = RN(1/den) for every significand), q = RN(x r), and ONE
// residual correction q + r (x - den q). hipcc's IEEE sequence applies the
// correction twice and adds the v_div_scale / v_div_fixup range steps; the
// second correction never changes the result - checked exhaustively on the
// GPU over all 2^46 significand pairs (scripts/probes/div_exhaustive.hip:
// 0 of 7.04e13 differ from x / den; profiles/r05_div_exhaustive.txt) - and
// the range steps only matter when a quotient, reciprocal or residual leaves
// the normal range, where the sequence is no longer scale-invariant. The
// guard keeps every intermediate normal: den in [2^-60, 2^60] (den is a pair
// distance clamped at 1e-12, so |x|, |y| <= den) and numerators zero or
// >= 2^-60 in magnitude; `ok` is cleared otherwise and the caller redoes the
// row with IEEE division. Branch-free, so consecutive pairs interleave.
// Also sampled against IEEE division: scripts/probes/fastmath_probe.hip.
__device__ __forceinline__ void div2_fast(float x, float y, float den, float *qx, float *qy,
                                          bool &ok)
{
    ok &= den >= 0x1p-60f && den <= 0x1p60f && mag_ok(x, 0x1p-60f, 0x1p60f) &&
          mag_ok(y, 0x1p-60f, 0x1p60f);
    float r = __builtin_amdgcn_rcpf(den);
    r = __builtin_fmaf(__builtin_fmaf(-den, r, 1.0f), r, r);
    const float q = x * r, p = y * r;
    *qx = __builtin_fmaf(__builtin_fmaf(-den, q, x), r, q);
    *qy = __builtin_fmaf(__builtin_fmaf(-den, p, y), r, p);
}

// acos of the bearing (environment.py:286): the device library's acosf
// (ROCm ocml: a degree-5 polynomial in r = |x| > 0.5 ? 0.5 - 0.5|x| : x*x,
// with a v_sqrt_f32 of r on the |x| > 0.5 branch). oracle/marlnav_oracle.c
// acos_device restates it op for op; the hardware sqrt, which is not
// correctly rounded, is restated from an exhaustive measurement of it on the
// only r that branch produces (k * 2^-25, tests/golden/vsqrt_r_grid.npz), so
// kernel and oracle bearings agree bit for bit (tests/golden/acos_dev_check.py
// checks every fp32 in [-1, 1]). MARLNAV_ACOS_CR_SQRT (A/B builds): the same
// sequence with the correctly rounded sqrt (sqrt_fast) - five more VALU per
// bearing, measured +0.24 us at 16384x3x3 and +0.32 us at 4096x16x32.
#ifndef MARLNAV_ACOS_CR_SQRT
#define MARLNAV_ACOS_CR_SQRT 0
#endif
__device__ __forceinline__ float acos_k(float x)
{
    if (!MARLNAV_ACOS_CR_SQRT) return acosf(x);
    const float ax = fabsf(x);
    const float rt = __builtin_fmaf(ax, -0.5f, 0.5f);
    const float x2 = x * x;
    const bool big = ax > 0.5f;
    const float r = big ? rt : x2;
    float p = __builtin_fmaf(__uint_as_float(0x3d1c21a7u), r, __uint_as_float(0x3c5fc5dau));
    p = __builtin_fmaf(r, p, __uint_as_float(0x3d034c3cu));
    p = __builtin_fmaf(r, p, __uint_as_float(0x3d3641b1u));
    p = __builtin_fmaf(r, p, __uint_as_float(0x3d999bc8u));
    p = __builtin_fmaf(r, p, __uint_as_float(0x3e2aaaacu));
    const float u = r * p;
    bool unused = true;
    const float sq = sqrt_fast(r, unused);
    const float s2 = __builtin_fmaf(sq, u, sq);
    const float zt = s2 + s2;
    const float ztn = __uint_as_float(0x40490fdbu) - zt;                      // pi - 2 asin(sqrt r)
    const float zs = __uint_as_float(0x3fc90fdbu) - __builtin_fmaf(x, u, x);  // pi/2 - asin(x)
    return big ? (x < 0.0f ? ztn : zt) : zs;
}

// The bearing of a normalised difference (nx, ny) seen from heading (dirx,
// diry): environment.py:280-286 (dot, clamp, x-residual sign, acos) and the
// dist < cap cap (:172-177).
template <bool FAST = false>
__device__ __forceinline__ float bearing_of(float nx, float ny, float dirx, float diry,
                                            float dist, float cap)
{
    float dot = dirx * nx + diry * ny;
    // FAST: dot is finite, so the clamp is one v_med3 (no compare/select
    // pairs and their VCC hazard nops); -0 passes through either way
    dot = FAST ? __builtin_amdgcn_fmed3f(dot, -1.0f, 1.0f) : clamp_t(dot, -1.0f, 1.0f);
    const float orth_x = nx - dot * dirx;
    const float ang = (orth_x > 0.0f ? -1.0f : 1.0f) * acos_k(dot);
    return dist < cap ? 0.0f : ang;
}

// _get_angles (environment.py:276-286) + the dist < 0.1 cap (:172-177).
// FAST: shared-reciprocal division (clears ok when it may differ from IEEE).
template <bool FAST = false>
__device__ __forceinline__ float pair_angle(float ox, float oy, float px, float py,
                                            float dirx, float diry, float dist, float cap,
                                            bool &ok)
{
    const float dx = px - ox, dy = py - oy;
    if (FAST && (MARLNAV_AB & 64)) return dx * dirx + dist;  // timing only: trivial pair math
    // F.normalize's clamp_min(1e-12). FAST (finite, non-negative dist): one
    // v_med3 instead of a canonicalize + v_max
    const float den = FAST ? __builtin_amdgcn_fmed3f(dist, 1e-12f, __builtin_inff())
                           : (dist > 1e-12f ? dist : 1e-12f);
    float nx, ny;
    if constexpr (FAST) {
        div2_fast(dx, dy, den, &nx, &ny, ok);
    } else {
        nx = dx / den;
        ny = dy / den;
    }
    return bearing_of<FAST>(nx, ny, dirx, diry, dist, cap);
}

// ------------------------------------------------- packed pair math (FAST)
// Two pairs of one row per instruction: the operations of pair_dist<true> +
// pair_angle<true> (and of the device acosf, op for op as acos_device in the
// oracle restates it) on (pair a, pair b) lanes of v_pk_add/mul/fma_f32,
// which take two fp32 operations per lane-slot where a VOP2 f32 instruction
// takes one. The per-element steps that have no packed form on gfx950
// (v_rsq/v_rcp/v_sqrt, v_max/v_med3, compares and selects) stay per element.
// Every packed operation is the same IEEE single operation per element as
// its scalar twin (no contraction: -ffp-contract=off, explicit fma), so the
// results are the scalar path's bits (scripts/probes/pair_forms.hip: 2^28
// random pair sets; the GPU suite: every kernel output against the oracle).
// No range guard: callers are coordinate-checked (FAST) blocks.
// Written with explicit .x/.y elements: the same math over generic W-wide
// clang vectors (W = 2, 4, 6) compiled to dependent packed instructions
// back to back, each pair of them separated by an s_nop, and measured
// slower (profiles/r06_pair_forms_widths.txt, r06_ab_packed_widths.txt).
typedef float f2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2_t pk_fma(f2_t a, f2_t b, f2_t c)
{
    return __builtin_elementwise_fma(a, b, c);
}

__device__ __forceinline__ f2_t f2s(float x) { return f2_t{x, x}; }

// the device library's acosf (ocml), op for op (acos_device in the oracle):
// r = |x| > 0.5 ? 0.5 - 0.5|x| : x*x; u = r P5(r); |x| <= 0.5: pi/2 - (x +
// x u); else 2(s + s u), or pi minus that for x < 0, s = v_sqrt_f32(r)
__device__ __forceinline__ f2_t acos2_dev(f2_t x)
{
    const f2_t ax = f2_t{__builtin_fabsf(x.x), __builtin_fabsf(x.y)};
    const f2_t rt = pk_fma(ax, f2s(-0.5f), f2s(0.5f));
    const f2_t x2 = x * x;
    const bool big0 = ax.x > 0.5f, big1 = ax.y > 0.5f;
    const f2_t r = f2_t{big0 ? rt.x : x2.x, big1 ? rt.y : x2.y};
    f2_t p = pk_fma(f2s(__uint_as_float(0x3d1c21a7u)), r, f2s(__uint_as_float(0x3c5fc5dau)));
    p = pk_fma(r, p, f2s(__uint_as_float(0x3d034c3cu)));
    p = pk_fma(r, p, f2s(__uint_as_float(0x3d3641b1u)));
    p = pk_fma(r, p, f2s(__uint_as_float(0x3d999bc8u)));
    p = pk_fma(r, p, f2s(__uint_as_float(0x3e2aaaacu)));
    const f2_t u = r * p;
    const f2_t sq = f2_t{__builtin_amdgcn_sqrtf(r.x), __builtin_amdgcn_sqrtf(r.y)};
    const f2_t s2 = pk_fma(sq, u, sq);
    const f2_t zt = s2 + s2;
    const f2_t ztn = f2s(__uint_as_float(0x40490fdbu)) - zt;
    const f2_t zs = f2s(__uint_as_float(0x3fc90fdbu)) - pk_fma(x, u, x);
    return f2_t{big0 ? (x.x < 0.0f ? ztn.x : zt.x) : zs.x, big1 ? (x.y < 0.0f ? ztn.y : zt.y) : zs.y};
}

// pair_dist<true> and pair_angle<true> of two pairs (px, py) of the row at
// (ox, oy) heading (dirx, diry): the distances and the capped bearings
__device__ __forceinline__ void pair2_fast(float ox, float oy, float dirx, float diry, f2_t px,
                                           f2_t py, float cap, f2_t &dist, f2_t &ang)
{
    const f2_t dx = px - f2s(ox), dy = py - f2s(oy);
    const f2_t q = pk_fma(dy, dy, dx * dx);
    // sqrt_fast: rsq, one FMA-residual correction, max(., 0)
    const f2_t y = f2_t{__builtin_amdgcn_rsqf(q.x), __builtin_amdgcn_rsqf(q.y)};
    const f2_t s = q * y, h = f2s(0.5f) * y;
    const f2_t e = pk_fma(-s, s, q);
    const f2_t t = pk_fma(e, h, s);
    dist = f2_t{__builtin_fmaxf(t.x, 0.0f), __builtin_fmaxf(t.y, 0.0f)};
    // F.normalize: den = max(dist, 1e-12), div2_fast
    const f2_t den = f2_t{__builtin_amdgcn_fmed3f(dist.x, 1e-12f, __builtin_inff()),
                          __builtin_amdgcn_fmed3f(dist.y, 1e-12f, __builtin_inff())};
    f2_t r = f2_t{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
    r = pk_fma(pk_fma(-den, r, f2s(1.0f)), r, r);
    const f2_t qx = dx * r, qy = dy * r;
    const f2_t nx = pk_fma(pk_fma(-den, qx, dx), r, qx);
    const f2_t ny = pk_fma(pk_fma(-den, qy, dy), r, qy);
    // bearing_of<true>
    f2_t dot = f2s(dirx) * nx + f2s(diry) * ny;
    dot = f2_t{__builtin_amdgcn_fmed3f(dot.x, -1.0f, 1.0f), __builtin_amdgcn_fmed3f(dot.y, -1.0f, 1.0f)};
    const f2_t orth = nx - dot * f2s(dirx);
    const f2_t ac = acos2_dev(dot);
    const float a0 = (orth.x > 0.0f ? -1.0f : 1.0f) * ac.x;
    const float a1 = (orth.y > 0.0f ? -1.0f : 1.0f) * ac.y;
    ang = f2_t{dist.x < cap ? 0.0f : a0, dist.y < cap ? 0.0f : a1};
}

// N pairs of one row (ox, oy, heading dirx, diry): pair2_fast on pairs
// (0, 1), (2, 3), ... and the scalar FAST pair math on an odd last one
template <int N>
__device__ __forceinline__ void pairs_fast(float ox, float oy, float dirx, float diry,
                                           const float (&px)[N], const float (&py)[N], float cap,
                                           float (&d)[N], float (&g)[N])
{
#pragma unroll
    for (int k = 0; k + 1 < N; k += 2) {
        f2_t d2, g2;
        pair2_fast(ox, oy, dirx, diry, f2_t{px[k], px[k + 1]}, f2_t{py[k], py[k + 1]}, cap, d2, g2);
        d[k] = d2.x;
        d[k + 1] = d2.y;
        g[k] = g2.x;
        g[k + 1] = g2.y;
    }
    if constexpr (N % 2 != 0) {
        bool unused = true;
        d[N - 1] = pair_dist<true>(ox, oy, px[N - 1], py[N - 1], unused);
        g[N - 1] = pair_angle<true>(ox, oy, px[N - 1], py[N - 1], dirx, diry, d[N - 1], cap, unused);
    }
}

// Correctly rounded fp32 sin/cos of an angle already clamped to [-pi, pi]
// (the heading update, environment.py:131-137). The reference evaluates
// torch.sin/cos on its CPU path, which in this torch build is MKL VML
// (vsSin/vsCos, <= 0.6 ulp, not correctly rounded); no fp32 sequence of ours
// can reproduce MKL's, and the correctly rounded value is the one that
// agrees with it most often (tests/golden/libm_check.py sweeps every fp32
// angle in [-pi, pi]: CR agrees with MKL on 95.1% of sines and cosines, the
// round-2 fp32 Cephes polynomials on 87-89%). Evaluated in fp64: two-part
// Cody-Waite reduction by pi/2 (|k| <= 2; k*PIO2_1 and x - k*PIO2_1 exact),
// the fdlibm __kernel_sin / __kernel_cos minimax polynomials on [-pi/4, pi/4]
// (error < 2^-58), one rounding to fp32 at the end. The sweep checks the
// result against a correctly rounded reference for every input of the range.
// NaN -> quadrant 0 (NaN propagates); sin(-0) = -0. The identical operation
// sequence (explicit FMAs, no contraction) is oracle_sincos in
// oracle/marlnav_oracle.c, so kernel and oracle agree bit for bit.
// A wave whose angles all lie in |th| < 0.78 (< pi/4: quadrant k = 0 on
// every lane, the common case) skips the reduction and the quadrant selects:
// the same operations on r = x, so the same bits.
__device__ __forceinline__ void sincos_k(float th, float *s_out, float *c_out)
{
    const double x = (double)th;
    if (MARLNAV_AB & 128) {  // timing only: no sin/cos
        *s_out = th;
        *c_out = 1.0f - th;
        return;
    }
    if (!(MARLNAV_AB & 32) && __ballot(!(fabsf(th) < 0.78f)) == 0ull) {
        const double z = x * x;
        double ps = __builtin_fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);
        ps = __builtin_fma(z, ps, 2.75573137070700676789e-06);
        ps = __builtin_fma(z, ps, -1.98412698298579493134e-04);
        ps = __builtin_fma(z, ps, 8.33333333332248946124e-03);
        ps = __builtin_fma(z, ps, -1.66666666666666324348e-01);
        const double sd = x == 0.0 ? x : __builtin_fma(z * x, ps, x);
        double pc = __builtin_fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);
        pc = __builtin_fma(z, pc, -2.75573143513906633035e-07);
        pc = __builtin_fma(z, pc, 2.48015872894767294178e-05);
        pc = __builtin_fma(z, pc, -1.38888888888741095749e-03);
        pc = __builtin_fma(z, pc, 4.16666666666666019037e-02);
        *s_out = (float)sd;
        *c_out = (float)__builtin_fma(z * z, pc, __builtin_fma(-0.5, z, 1.0));
        return;
    }
    const double k = __builtin_rint(x * 6.36619772367581382433e-01);
    double r = __builtin_fma(-k, 1.57079632673412561417e+00, x);
    r = __builtin_fma(-k, 6.07710050650619224932e-11, r);
    r = k == 0.0 ? x : r;  // keeps the sign of -0
    const double z = r * r;
    double ps = __builtin_fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);
    ps = __builtin_fma(z, ps, 2.75573137070700676789e-06);
    ps = __builtin_fma(z, ps, -1.98412698298579493134e-04);
    ps = __builtin_fma(z, ps, 8.33333333332248946124e-03);
    ps = __builtin_fma(z, ps, -1.66666666666666324348e-01);
    const double sd = r == 0.0 ? r : __builtin_fma(z * r, ps, r);  // sin(-0) = -0
    double pc = __builtin_fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);
    pc = __builtin_fma(z, pc, -2.75573143513906633035e-07);
    pc = __builtin_fma(z, pc, 2.48015872894767294178e-05);
    pc = __builtin_fma(z, pc, -1.38888888888741095749e-03);
    pc = __builtin_fma(z, pc, 4.16666666666666019037e-02);
    const double cd = __builtin_fma(z * z, pc, __builtin_fma(-0.5, z, 1.0));
    const float sn = (float)sd, cs = (float)cd;
    const bool q1 = k == 1.0, q3 = k == -1.0, q2 = k == 2.0 || k == -2.0;
    *s_out = q1 ? cs : (q3 ? -cs : (q2 ? -sn : sn));
    *c_out = q1 ? -sn : (q3 ? sn : (q2 ? -cs : cs));
}

// ----------------------------------------------------------- native RNG
// The native stream (rng='native'; a distributional match of the reference's
// torch.rand draws, utils.py:381-398, checked by tests/test_native_rng_dist.py):
// Philox2x32-10 (Salmon et al., SC'11: Random123's philox2x32 at its default
// 10 rounds; its published known-answer vectors are checked in
// tests/test_oracle_golden.py). Uniform #idx of env gid at step s is word
// idx & 1 of block idx >> 1: counter (lo32(gid), lo32(s) ^ hi32(gid) *
// 0x85EBCA77) under the key native_key(seed, idx >> 1, s), on torch.rand's
// 24-bit grid. The key holds no per-env term, so where the block index is
// wave-uniform (the env-block kernel's draws) it and its round increments
// live in SGPRs. Obstacle j is block j (x = word 0, y = word 1): one block per
// obstacle, so an A3/O3 env block draws exactly one block per thread
// (Philox4x32-10, rounds 1-4, drew two 4-word blocks per env on two of the
// three waves: 20 v_mad_u64_u32 per drawing lane against 10 here).
// oracle/marlnav_oracle.c restates it.
constexpr uint32_t kPhiloxM2 = 0xD256D193u, kPhiloxW = 0x9E3779B9u;

__device__ __forceinline__ void philox2x32_10(uint32_t &c0, uint32_t &c1, uint32_t k)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one v_mad_u64_u32 per round for the 64-bit product
        const uint64_t p = (uint64_t)c0 * kPhiloxM2;
        const uint32_t hi = (uint32_t)(p >> 32), lo = (uint32_t)p;
        c0 = __builtin_amdgcn_bitop3_b32(hi, k, c1, 0x96);  // hi ^ k ^ c1 in one VALU
        c1 = lo;
        k += kPhiloxW;
    }
}

// The caller's 64-bit seed enters the stream only through its splitmix64
// finalisation (Steele, Lea, Flood, OOPSLA'14: a bijection of the 64-bit
// words), done once per launch on the host (marlnav_step, marlnav_reinit_all
// store it in the kernel's MarlnavParams.seed): seeds that differ in either
// word give unrelated mixed seeds.
__host__ __device__ constexpr uint64_t native_seed_mix(uint64_t seed)
{
    uint64_t z = seed + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// murmur3's 32-bit finaliser (a bijection)
__host__ __device__ constexpr uint32_t fmix32(uint32_t h)
{
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    return h ^ (h >> 16);
}

// the 32-bit Philox key of block `blk` at step s from the MIXED seed m
// (native_seed_mix): its low word XOR fmix32 of the block index, the high
// word of s (zero below 2^32 steps) and m's high word. No linear relation
// ties (seed, blk) to (seed', blk'): a key shared by two of them is a
// 2^-32 coincidence of the hashes, not a shift of the block index. The
// counter carries the env id and the low word of s. Where blk is
// wave-uniform (the env-block kernel's draws) the key is SALU work.
__host__ __device__ constexpr uint32_t native_key(uint64_t m, uint32_t blk, uint64_t s)
{
    return (uint32_t)m ^
           fmix32(blk * 0x9E3779B1u + (uint32_t)(s >> 32) * 0x85EBCA77u + (uint32_t)(m >> 32));
}

// block `blk` of env gid at step s: two 32-bit words
__device__ __forceinline__ void native_block(uint64_t seed, uint32_t blk, uint64_t gid, uint64_t s,
                                             uint32_t &r0, uint32_t &r1)
{
    r0 = (uint32_t)gid;
    r1 = (uint32_t)s ^ ((uint32_t)(gid >> 32) * 0x85EBCA77u);
    if (!(MARLNAV_AB & 4)) philox2x32_10(r0, r1, native_key(seed, blk, s));  // (AB 4: timing only)
}

// a 32-bit word -> [0, 1) on a 24-bit grid (torch.rand's fp32 values)
__device__ __forceinline__ float native_u24(uint32_t r) { return (float)(r >> 8) * 0x1.0p-24f; }

// uniform #idx of env gid at step s
__device__ __forceinline__ float native_uniform(uint64_t seed, uint64_t gid, uint64_t s,
                                                uint32_t idx)
{
    uint32_t r0, r1;
    native_block(seed, idx >> 1, gid, s, r0, r1);
    return native_u24((idx & 1u) ? r1 : r0);
}

// obstacle j of env gid at step s, scaled like the reference's sampler
// (utils.py:390-398): v[0] = x, v[1] = y
__device__ __forceinline__ void native_obst_draw(uint64_t seed, uint64_t s, uint64_t gid, int j,
                                                 float rx, float mx, float ry, float my, float v[2])
{
    uint32_t r0, r1;
    native_block(seed, (uint32_t)j, gid, s, r0, r1);
    v[0] = rx * (native_u24(r0) - 0.5f) + mx;
    v[1] = ry * (native_u24(r1) - 0.5f) + my;
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
    for (int j = 0; j < S; ++j) {  // one Philox block per obstacle
        float v[2];
        native_obst_draw(pr.seed, sidx, gid, j, pr.obs_range_x, pr.obs_mean_x, pr.obs_range_y,
                         pr.obs_mean_y, v);
        put(ob + 2 * j, v[0]);
        put(ob + 2 * j + 1, v[1]);
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
                                           const float *__restrict__ scale, int D, bool wt)
{
    int head = 0;
    const OutBuf ob = out_buf(dst, 4u * n);
    wt = kWtOut && wt;
    if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
        const int n4 = n >> 2;
        for (int i = lane; i < n4; i += 64) {
            const float4 v = *reinterpret_cast<const float4 *>(src + 4 * i);
            if (wt)
                wt_st4(ob, 16u * i, v);
            else
                out_st4(dst + 4 * i, v);
        }
        head = n4 << 2;
    }
    for (int i = head + lane; i < n; i += 64) {
        if (wt)
            wt_st(ob, 4u * i, src[i]);
        else
            out_st(dst + i, src[i]);
    }
    if (nrm_dst) {
        const OutBuf nb = out_buf(nrm_dst, 4u * n);
        for (int i = lane; i < n; i += 64) {
            const int k = i % D;
            const float v = (src[i] - mean[k]) / scale[k];
            if (wt)
                wt_st(nb, 4u * i, v);
            else
                nrm_dst[i] = v;
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

// _bond_reward's per-distance term (environment.py:264-269), 1 / (1 + sd^2)
// with sd = (d - ideal) / sharpness. FAST (kTermsFastFlag set: every
// parameter inside the short sequences' guards, FAST coordinates): the exact
// short division and reciprocal; REFC: sharpness == 1, the division dropped.
template <bool FAST, bool REFC = false>
__device__ __forceinline__ float bond_term(float d, const MarlnavParams &pr, bool &ok)
{
    if constexpr (FAST) {
        if constexpr (REFC) {
            const float sd = d - pr.ideal_dist;
            return recip_fast(1.0f + sd * sd, ok);
        } else {
            const DivC d_sharp = make_divc(pr.bond_sharpness, ok);
            const float sd = div_c(d - pr.ideal_dist, d_sharp, ok);
            return recip_fast(1.0f + sd * sd, ok);
        }
    } else {
        const float sd = (d - pr.ideal_dist) / pr.bond_sharpness;
        return 1.0f / (1.0f + sd * sd);
    }
}

// The per-agent reward of _rews_and_terms (environment.py:184-269) for one
// row, from its target bearing/distance, risk and collision flags, the count
// of others in the distance band and the torch-order sum of bond terms.
template <int A, bool FAST, bool REFC>
__device__ __forceinline__ RowOut row_reward(float ta, float td, bool risk_any, bool col_any,
                                             float band, float bond, const MarlnavParams &pr,
                                             bool &ok)
{
    const float head = fabsf(ta) < pr.max_angle_diff ? 1.0f : 0.0f;
    const float bandc = band < pr.max_at_prop_d ? band : pr.max_at_prop_d;
    float dsc, soft;
    if (FAST && (pr.flags & kTermsFastFlag)) {
        // exact: the host set kTermsFastFlag only for parameters inside the
        // div_c / recip_fast guards (terms_fast_params), and FAST coordinates
        // bound every distance (coord_ok), so every operand stays in range
        const DivC d_init = make_divc(pr.init_dist, ok);
        soft = -1.0f * div_c(td, d_init, ok);
        if constexpr (REFC) {
            dsc = bandc * 0.5f;
        } else {
            const DivC d_mapd = make_divc(pr.max_at_prop_d, ok);
            dsc = div_c(bandc, d_mapd, ok);
        }
    } else {
        dsc = bandc / pr.max_at_prop_d;
        soft = -1.0f * (td / pr.init_dist);
    }
    const float bondm = bond / (float)(A - 1);  // the bond sum can be tiny: IEEE
    const float risk = risk_any ? 1.0f : 0.0f;
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
    return RowOut{rm, rh, (col_any ? 1u : 0u) | ((td < pr.target_radius) ? 2u : 0u)};
}

// observe_row with compile-time shape and the packed row kept in registers
// (row[D]); others are visited as j = 0..A-2 -> agent j + (j >= a), so
// every row index is a compile-time constant.
// The own row (ox, oy, dx, dy) comes in registers; the env's other agents
// are read from sts.
// REFC: the reference's own constants bond_sharpness == 1 and
// max_at_prop_d == 2 (environment.py:62, 66): (d - ideal) / 1 is d - ideal and
// band / 2 is band * 0.5 exactly, so those two divisions are dropped (a
// separate instance, chosen per launch by the caller).
template <int A, int O, bool TERMS, bool FAST, bool REFC = false>
__device__ __forceinline__ RowOut observe_row_own(const float *__restrict__ sts,
                                                  const float *__restrict__ obe,
                                                  const float *__restrict__ tge, int a,
                                                  float ox, float oy, float dx, float dy,
                                                  float *row, const MarlnavParams &pr, bool &ok)
{
    const float cap = pr.cap_distance;
    if constexpr (FAST && MARLNAV_PACKED_PAIRS && !(MARLNAV_AB & 64)) {
        // the row's pairs in row order - target, obstacles, other agents -
        // two per pair2_fast (the same bits as pair_dist/pair_angle<true>,
        // scripts/probes/pair_forms.hip); an odd last pair alone
        constexpr int NP = 1 + O + (A - 1);
        float px[NP], py[NP], pd[NP], pg[NP];
        px[0] = tge[0];
        py[0] = tge[1];
#pragma unroll
        for (int j = 0; j < O; ++j) {
            px[1 + j] = obe[2 * j];
            py[1 + j] = obe[2 * j + 1];
        }
#pragma unroll
        for (int j = 0; j < A - 1; ++j) {
            const int m = j + (j >= a ? 1 : 0);
            px[1 + O + j] = sts[5 * m];
            py[1 + O + j] = sts[5 * m + 1];
        }
        pairs_fast<NP>(ox, oy, dx, dy, px, py, cap, pd, pg);
        row[0] = pg[0];
        row[1] = pd[0];
        bool ob_risk = false, ob_col = false, ag_risk = false, ag_col = false;
        float band = 0.0f;
#pragma unroll
        for (int j = 0; j < O; ++j) {
            row[2 + j] = pg[1 + j];
            row[2 + O + j] = pd[1 + j];
            if (TERMS) {
                ob_risk |= pd[1 + j] < pr.ob_risk_dist;
                ob_col |= pd[1 + j] < pr.ob_coll_dist;
            }
        }
#pragma unroll
        for (int j = 0; j < A - 1; ++j) {
            const float d = pd[1 + O + j];
            row[2 + 2 * O + j] = pg[1 + O + j];
            row[2 + 2 * O + (A - 1) + j] = d;
            if (TERMS) {
                ag_risk |= d < pr.ag_risk_dist;
                ag_col |= d < pr.ag_coll_dist;
                band += (pr.agents_min_d < d && d < pr.agents_max_d) ? 1.0f : 0.0f;
            }
        }
        RowOut out{0.0f, 0.0f, 0u};
        if (TERMS) {
            const float *agd = row + 2 + 2 * O + (A - 1);
            float bond;
            if (pr.flags & kTermsFastFlag)
                bond = torch_row_sum_r<A - 1>(agd, [&](float d) { return bond_term<true, REFC>(d, pr, ok); });
            else
                bond = torch_row_sum_r<A - 1>(agd, [&](float d) { return bond_term<false>(d, pr, ok); });
            out = row_reward<A, FAST, REFC>(pg[0], pd[0], ob_risk || ag_risk, ob_col || ag_col, band,
                                            bond, pr, ok);
        }
        return out;
    }
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
        const float *agd = row + 2 + 2 * O + (A - 1);  // the others_distances just written
        float bond;
        if (FAST && (pr.flags & kTermsFastFlag))
            bond = torch_row_sum_r<A - 1>(agd, [&](float d) { return bond_term<true, REFC>(d, pr, ok); });
        else
            bond = torch_row_sum_r<A - 1>(agd, [&](float d) { return bond_term<false>(d, pr, ok); });
        out = row_reward<A, FAST, REFC>(ta, td, ob_risk || ag_risk, ob_col || ag_col, band, bond, pr,
                                        ok);
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
__device__ __forceinline__ void store_row(float *__restrict__ dst, const float *row, bool wt)
{
    if (kWtOut && wt) {
        // per-lane row pointers: one written-through buffer from the first
        // active lane's row
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)(uintptr_t)dst >> 32));
        float *b0 = reinterpret_cast<float *>(((uint64_t)hi << 32) | lo);
        const OutBuf ob = out_buf(b0, 1u << 26);
        const uint32_t off = (uint32_t)((const char *)dst - (const char *)b0);
        if constexpr (D % 4 == 0) {
#pragma unroll
            for (int k = 0; k < D; k += 4)
                wt_st4(ob, off + 4u * k, make_float4(row[k], row[k + 1], row[k + 2], row[k + 3]));
        } else if constexpr (D % 2 == 0) {
#pragma unroll
            for (int k = 0; k < D; k += 2) wt_st2(ob, off + 4u * k, make_float2(row[k], row[k + 1]));
        } else {
#pragma unroll
            for (int k = 0; k < D; ++k) wt_st(ob, off + 4u * k, row[k]);
        }
    } else if constexpr (D % 4 == 0) {
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
