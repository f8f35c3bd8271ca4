// marlnav_step.hip - gfx950 (MI355X) kernels behind include/marlnav.h.
//
// One launch performs the whole Env.step of the reference
// (marlnav/environment.py:92-107): heading/speed integration, every
// agent->target/obstacle/agent distance and bearing, the reward terms, the
// terminal logic, the masked re-initialisation of finished envs and the
// recomputed observations of those envs.
//
// Mapping: a workgroup owns a tile of E consecutive envs and
// runs one lane per agent row (R = E*A lanes, env-major, so lane t owns row
// e0*A + t of the (P*A, .) agent arrays). The tile's array-of-structs inputs
// (states 5A floats/env, obstacles 2S, target 2) are staged in LDS with
// 16-byte coalesced loads; the packed observation tile (A*D floats/env) is
// assembled in LDS and streamed out with 16-byte coalesced stores. Per-env
// reductions over agents go through LDS. No MFMA: nothing here contracts.
//
// Numerics: built with -ffp-contract=off and the HIP default
// correctly rounded fp32 division and sqrt, so every distance, dot product
// and reward term is the same fp32 expression the reference's CPU path
// evaluates. The heading rotation evaluates sin/cos in double and rounds once
// (see oracle/marlnav_oracle.c for the identical CPU recipe); acos is the
// device libm's acosf.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/marlnav.h"

namespace {

constexpr float kPiF = 3.14159265358979323846f;

// Timing-only ablation builds (scripts/kbench.py; never shipped, results
// wrong by construction): 1 no acos, 2 fast fp32 sin/cos, 4 fast division,
// 8 fast sqrt, 16 no observation math at all.
#ifndef MARLNAV_ABLATE
#define MARLNAV_ABLATE 0
#endif

// Diagnostic build (MARLNAV_STAMPS=1, scripts/kstamps.py): lane 0 of every
// block records s_memrealtime / s_memtime at each phase boundary into a
// buffer registered with marlnav_debug_stamps(). Never in the shipped build.
#ifndef MARLNAV_STAMPS
#define MARLNAV_STAMPS 0
#endif
#if MARLNAV_STAMPS
__device__ unsigned long long *g_stamps;
#define STAMP(k)                                                                   \
    do {                                                                           \
        if (threadIdx.x == 0) {                                                    \
            unsigned long long *sp_ = g_stamps + (size_t)blockIdx.x * 16;          \
            sp_[2 * (k)] = wall_clock64();                                         \
            sp_[2 * (k) + 1] = clock64();                                          \
        }                                                                          \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif
constexpr int kMaxAgents = 64;
constexpr int kMaxStride = 256;
constexpr int kLdsBudget = 48 * 1024;

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

__host__ __device__ inline int obs_dim(int A, int O) { return 2 + 2 * O + 2 * (A - 1); }

// ------------------------------------------------------------- device math
__device__ __forceinline__ float clamp_t(float x, float lo, float hi)
{
    x = x < lo ? lo : x;  // NaN passes through like torch.clamp
    return x > hi ? hi : x;
}

// torch.cdist direct path (environment.py:271-274)
__device__ __forceinline__ float pair_dist(float ox, float oy, float px, float py)
{
    const float dx = px - ox, dy = py - oy;
#if MARLNAV_ABLATE & 8
    return __builtin_amdgcn_sqrtf(__builtin_fmaf(dy, dy, dx * dx));
#else
    return __builtin_sqrtf(__builtin_fmaf(dy, dy, dx * dx));
#endif
}

// _get_angles (environment.py:276-286) + the dist < 0.1 cap (:172-177)
__device__ __forceinline__ float pair_angle(float ox, float oy, float px, float py,
                                            float dirx, float diry, float dist, float cap)
{
    const float dx = px - ox, dy = py - oy;
    const float den = dist > 1e-12f ? dist : 1e-12f;
#if MARLNAV_ABLATE & 4
    const float nx = __fdividef(dx, den), ny = __fdividef(dy, den);
#else
    const float nx = dx / den, ny = dy / den;
#endif
    float dot = dirx * nx + diry * ny;
    dot = clamp_t(dot, -1.0f, 1.0f);
    const float orth_x = nx - dot * dirx;
#if MARLNAV_ABLATE & 1
    const float ang = (orth_x > 0.0f ? -1.0f : 1.0f) * dot;
#else
    const float ang = (orth_x > 0.0f ? -1.0f : 1.0f) * acosf(dot);
#endif
    return dist < cap ? 0.0f : ang;
}

__device__ __forceinline__ void sincos_rn(float th, float *s, float *c)
{
#if MARLNAV_ABLATE & 2
    __sincosf(th, s, c);
#else
    double sd, cd;
    sincos((double)th, &sd, &cd);
    *s = (float)sd;
    *c = (float)cd;
#endif
}

// ----------------------------------------------------------- native RNG
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c[0], hi0 = __umulhi(0xD2511F53u, c[0]);
        const uint32_t lo1 = 0xCD9E8D57u * c[2], hi1 = __umulhi(0xCD9E8D57u, c[2]);
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

// native TriangleIntitializer draw for one env (utils.py:375-398)
__device__ void native_fresh_env(int A, int S, const MarlnavParams &pr,
                                 const float *__restrict__ formation, uint64_t gid,
                                 uint64_t sidx, float *st, float *ob, float *tg)
{
    for (int j = 0; j < S; ++j) {
        const float ux = native_uniform(pr.seed, gid, sidx, (uint32_t)(2 * j));
        const float uy = native_uniform(pr.seed, gid, sidx, (uint32_t)(2 * j + 1));
        ob[2 * j] = pr.obs_range_x * (ux - 0.5f) + pr.obs_mean_x;
        ob[2 * j + 1] = pr.obs_range_y * (uy - 0.5f) + pr.obs_mean_y;
    }
    for (int i = 0; i < 5 * A; ++i) st[i] = formation[i];
    tg[0] = formation[5 * A];
    tg[1] = formation[5 * A + 1];
    if (pr.flags & MARLNAV_NOISY_AGENTS) {
        const uint32_t base = (uint32_t)(2 * S);
        for (int i = 0; i < A; ++i) {
            const float u1 = native_uniform(pr.seed, gid, sidx, base + 3 * i);
            const float u2 = native_uniform(pr.seed, gid, sidx, base + 3 * i + 1);
            const float u3 = native_uniform(pr.seed, gid, sidx, base + 3 * i + 2);
            const double rad = sqrt(-2.0 * log(1.0 - (double)u1));
            const double ang = 6.283185307179586 * (double)u2;
            const float z0 = (float)(rad * cos(ang)), z1 = (float)(rad * sin(ang));
            float *s = st + 5 * i;
            s[0] = s[0] + pr.ags_dist * (pr.noise_std * z0);
            s[1] = s[1] + pr.ags_dist * (pr.noise_std * z1);
            float sn, c;
            sincos_rn(pr.angle_range * (u3 - 0.5f), &sn, &c);
            const float dx = s[2], dy = s[3];
            s[2] = c * dx + (-sn) * dy;
            s[3] = sn * dx + c * dy;
        }
    }
}

// ------------------------------------------------------------ tile copies
// Cooperative contiguous copy of n floats, 16-byte vectors where both sides
// allow it. LDS destinations are 16-byte aligned by construction.
__device__ __forceinline__ void tile_load(float *__restrict__ dst, const float *__restrict__ src,
                                          int n, int tid, int nthr)
{
    int head = 0;
    if ((reinterpret_cast<uintptr_t>(src) & 15u) == 0) {
        const int n4 = n >> 2;
        const float4 *s4 = reinterpret_cast<const float4 *>(src);
        float4 *d4 = reinterpret_cast<float4 *>(dst);
        for (int i = tid; i < n4; i += nthr) d4[i] = s4[i];
        head = n4 << 2;
    }
    for (int i = head + tid; i < n; i += nthr) dst[i] = src[i];
}

__device__ __forceinline__ void tile_store(float *__restrict__ dst, const float *__restrict__ src,
                                           int n, int tid, int nthr)
{
    int head = 0;
    if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
        const int n4 = n >> 2;
        const float4 *s4 = reinterpret_cast<const float4 *>(src);
        float4 *d4 = reinterpret_cast<float4 *>(dst);
        for (int i = tid; i < n4; i += nthr) d4[i] = s4[i];
        head = n4 << 2;
    }
    for (int i = head + tid; i < n; i += nthr) dst[i] = src[i];
}

// Stage three contiguous global ranges into LDS with every global load of
// the tile issued before the first wait: up to KMAX 16-byte vectors per
// lane are held in registers, then written to LDS. (A load -> LDS-store ->
// next-load loop would pay one full memory round trip per iteration.)
struct Span {
    const float *src;
    float *dst;
    int n;  // floats
};

template <int KMAX>
__device__ __forceinline__ void stage_spans(Span a, Span b, Span c, int tid, int nthr)
{
    const bool vec = ((reinterpret_cast<uintptr_t>(a.src) | reinterpret_cast<uintptr_t>(b.src) |
                       reinterpret_cast<uintptr_t>(c.src)) & 15u) == 0 && nthr >= 12;
    if (!vec) {  // unaligned shard base: plain scalar staging
        tile_load(a.dst, a.src, a.n, tid, nthr);
        tile_load(b.dst, b.src, b.n, tid, nthr);
        tile_load(c.dst, c.src, c.n, tid, nthr);
        return;
    }
    const int va = a.n >> 2, vb = b.n >> 2, vc = c.n >> 2;
    const int vt = va + vb + vc;
    float4 r[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int i = tid + k * nthr;
        if (i < vt) {
            const float *p = i < va ? a.src + 4 * i
                                    : (i < va + vb ? b.src + 4 * (i - va) : c.src + 4 * (i - va - vb));
            r[k] = *reinterpret_cast<const float4 *>(p);
        }
    }
    // scalar tails (< 4 floats per span), one lane per float
    float t = 0.0f;
    const int ta = a.n & 3, tb = b.n & 3, tc = c.n & 3;
    const int lane_t = tid - (nthr - 12);  // last 12 lanes take the tails
    const float *tsrc = nullptr;
    float *tdst = nullptr;
    if (lane_t >= 0) {
        const int j = lane_t & 3, w = lane_t >> 2;
        const Span &sp = w == 0 ? a : (w == 1 ? b : c);
        const int tn = w == 0 ? ta : (w == 1 ? tb : tc);
        if (j < tn) {
            tsrc = sp.src + (sp.n & ~3) + j;
            tdst = sp.dst + (sp.n & ~3) + j;
            t = *tsrc;
        }
    }
    // generic tiles with more vectors than KMAX per lane
    for (int i = tid + KMAX * nthr; i < vt; i += nthr) {
        const float *p = i < va ? a.src + 4 * i
                                : (i < va + vb ? b.src + 4 * (i - va) : c.src + 4 * (i - va - vb));
        float *q = i < va ? a.dst + 4 * i
                          : (i < va + vb ? b.dst + 4 * (i - va) : c.dst + 4 * (i - va - vb));
        *reinterpret_cast<float4 *>(q) = *reinterpret_cast<const float4 *>(p);
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int i = tid + k * nthr;
        if (i < vt) {
            float *q = i < va ? a.dst + 4 * i
                              : (i < va + vb ? b.dst + 4 * (i - va) : c.dst + 4 * (i - va - vb));
            *reinterpret_cast<float4 *>(q) = r[k];
        }
    }
    if (tdst) *tdst = t;
}

// ObsNormalizer fused into the store (utils.py:530-532)
__device__ __forceinline__ void tile_store_norm(float *__restrict__ dst,
                                                const float *__restrict__ src, int n, int D,
                                                const float *__restrict__ mean,
                                                const float *__restrict__ scale, int tid, int nthr)
{
    for (int i = tid; i < n; i += nthr) {
        const int k = i % D;
        dst[i] = (src[i] - mean[k]) / scale[k];
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

// ------------------------------------------------------------ row observe
struct RowOut {
    float r_miss, r_hit;  // agent reward if the env misses / reaches the target
    unsigned flags;       // bit0: obstacle or agent collision, bit1: in target
};

// observations() for agent row `a` of one env (environment.py:139-180), with
// the per-agent reward terms of _rews_and_terms (:184-269) when TERMS.
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
    const float ta = pair_angle(ox, oy, tx, ty, dx, dy, td, cap);
    row[0] = ta;
    row[1] = td;

    bool ob_risk = false, ob_col = false;
#pragma unroll
    for (int j = 0; j < O; ++j) {
        const float px = obe[2 * j], py = obe[2 * j + 1];
        const float d = pair_dist(ox, oy, px, py);
        row[2 + j] = pair_angle(ox, oy, px, py, dx, dy, d, cap);
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
        ang_out[k] = pair_angle(ox, oy, px, py, dx, dy, d, cap);
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

// -------------------------------------------------------------- LDS plan
struct TilePlan {
    int E, R, A, O, S, D;
    int off_st, off_ob, off_tg, off_obs, off_rm, off_rh, off_fl, off_env, off_cnt, off_nm,
        off_ns;
    int bytes;
};

__host__ __device__ inline int align4(int n) { return (n + 3) & ~3; }  // floats -> 16 B

__host__ __device__ inline TilePlan make_plan(int E, int A, int O, int S)
{
    TilePlan p;
    p.E = E;
    p.A = A;
    p.O = O;
    p.S = S;
    p.R = E * A;
    p.D = obs_dim(A, O);
    int o = 0;
    p.off_st = o;  o += align4(p.R * 5);
    p.off_ob = o;  o += align4(E * S * 2);
    p.off_tg = o;  o += align4(E * 2);
    p.off_obs = o; o += align4(p.R * p.D);
    p.off_rm = o;  o += align4(p.R);
    p.off_rh = o;  o += align4(p.R);
    p.off_fl = o;  o += align4(p.R);
    p.off_env = o; o += align4(E);
    p.off_cnt = o; o += 4;
    p.off_nm = o;  o += align4(p.D);
    p.off_ns = o;  o += align4(p.D);
    p.bytes = o * 4;
    return p;
}

struct StepArgs {
    MarlnavStepBuffers b;
    int64_t P;
    int64_t env_offset;
    int64_t slots;
    uint64_t step_idx;
    int E, A, O, S;
};

// env-level bits kept in LDS between phases
constexpr unsigned kFin = 1u;

// --------------------------------------------------------------- step kernel
template <int A_T, int O_T>
__global__ void __launch_bounds__(1024) step_kernel(StepArgs args, MarlnavParams pr)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int A = A_T ? A_T : args.A;
    const int O = O_T ? O_T : args.O;
    const int S = args.S;
    const TilePlan tp = make_plan(args.E, A, O, S);
    const int E = tp.E, D = tp.D;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * E;
    const int ne = (int)((args.P - e0) < E ? (args.P - e0) : E);
    const int nr = ne * A;

    float *st = lds + tp.off_st;
    float *ob = lds + tp.off_ob;
    float *tg = lds + tp.off_tg;
    float *obs = lds + tp.off_obs;
    float *rmiss = lds + tp.off_rm;
    float *rhit = lds + tp.off_rh;
    unsigned *rfl = reinterpret_cast<unsigned *>(lds + tp.off_fl);
    unsigned *envbits = reinterpret_cast<unsigned *>(lds + tp.off_env);
    unsigned *cnt = reinterpret_cast<unsigned *>(lds + tp.off_cnt);
    const MarlnavStepBuffers &b = args.b;
    const bool norm = (pr.flags & MARLNAV_WRITE_OBS_NORM) != 0;

    STAMP(0);
    // ---- phase 0: stage the tile (all global loads in flight together)
    float2 act = make_float2(0.0f, 0.0f);
    if (tid < nr) act = reinterpret_cast<const float2 *>(b.actions)[e0 * A + tid];
    float step_num_in = 0.0f;
    uint8_t term_in = 0;
    if (tid < ne) {
        step_num_in = b.step_num[e0 + tid];
        term_in = b.terminates[e0 + tid];
    }
    stage_spans<4>(Span{b.states + e0 * A * 5, st, nr * 5},
                   Span{b.obstacles + e0 * S * 2, ob, ne * S * 2},
                   Span{b.target + e0 * 2, tg, ne * 2}, tid, nthr);
    if (norm) {
        for (int k = tid; k < D; k += nthr) {
            lds[tp.off_nm + k] = b.norm_mean[k];
            lds[tp.off_ns + k] = b.norm_scale[k];
        }
    }
    if (tid < 3) cnt[tid] = 0u;
    __syncthreads();
    STAMP(1);

    // ---- phase 1: _move_agents (environment.py:113-123)
    const int el = tid / A, a = tid - el * A;
    if (tid < nr) {
        float a0 = act.x, a1 = act.y;
        if (pr.flags & MARLNAV_SCALE_ACTIONS) {  // ActionScaler (utils.py:546-547)
            a0 = pr.act_scale[0] * a0 + pr.act_mean[0];
            a1 = pr.act_scale[1] * a1 + pr.act_mean[1];
        }
        float *s = st + 5 * tid;
        float sn, c;
        sincos_rn(clamp_t(a0, -kPiF, kPiF), &sn, &c);
        const float dx = s[2], dy = s[3];
        const float ndx = c * dx + (-sn) * dy;
        const float ndy = sn * dx + c * dy;
        const float v = clamp_t(s[4] + clamp_t(a1, pr.min_accel, pr.max_accel), pr.min_speed,
                                pr.max_speed);
        s[0] = s[0] + ndx * v;
        s[1] = s[1] + ndy * v;
        s[2] = ndx;
        s[3] = ndy;
        s[4] = v;
    }
    __syncthreads();
    STAMP(2);

    // ---- phase 2: observations of the moved state + reward terms (:99-100)
    if (tid < nr && !(MARLNAV_ABLATE & 16)) {
        const RowOut ro = observe_row<A_T, O_T, true>(A, O, st + 5 * A * el, ob + 2 * S * el,
                                                      tg + 2 * el, a, obs + tid * D, pr);
        rmiss[tid] = ro.r_miss;
        rhit[tid] = ro.r_hit;
        rfl[tid] = ro.flags;
    }
    __syncthreads();
    STAMP(3);

    // ---- phase 3: per-env reductions, terminal logic, masked re-init
    if (tid < ne) {
        const int64_t e = e0 + tid;
        unsigned any_col = 0u, all_in = 1u;
        for (int i = 0; i < A; ++i) {
            const unsigned f = rfl[tid * A + i];
            any_col |= f & 1u;
            all_in &= (f >> 1) & 1u;
        }
        const float *rr = all_in ? rhit : rmiss;
        const float rsum = torch_row_sum(rr + tid * A, A, [](float r) { return r; });
        b.reward[e] = rsum / (float)A;                     // torch.mean (:233)

        float step_num = step_num_in + 1.0f;               // :96
        const bool truncated = step_num > pr.trunc_after;  // :97
        const bool term_old = term_in != 0;
        const bool terminated = any_col || term_old;       // :213-214
        b.terminates[e] = (uint8_t)(!term_old && all_in);  // :218-219
        b.terminated[e] = (uint8_t)terminated;
        b.truncated[e] = (uint8_t)truncated;
        if (truncated) atomicAdd(&cnt[0], 1u);
        if (any_col) atomicAdd(&cnt[1], 1u);
        if (all_in) atomicAdd(&cnt[2], 1u);

        unsigned bits = 0u;
        if (truncated || terminated) {                     // :102-104
            bits = kFin;
            float *sts = st + 5 * A * tid;
            float *obe = ob + 2 * S * tid;
            float *tge = tg + 2 * tid;
            if (b.fresh_states) {
                if (!(pr.flags & MARLNAV_FRESH_STATES_FROM_MOVED))
                    for (int i = 0; i < 5 * A; ++i) sts[i] = b.fresh_states[e * A * 5 + i];
                for (int i = 0; i < 2 * S; ++i) obe[i] = b.fresh_obstacles[e * S * 2 + i];
                tge[0] = b.fresh_target[2 * e];
                tge[1] = b.fresh_target[2 * e + 1];
            } else {
                native_fresh_env(A, S, pr, b.formation, (uint64_t)(args.env_offset + e),
                                 args.step_idx, sts, obe, tge);
            }
            for (int i = 0; i < 2 * S; ++i) b.obstacles[e * S * 2 + i] = obe[i];
            b.target[2 * e] = tge[0];
            b.target[2 * e + 1] = tge[1];
            step_num = 0.0f;
        }
        b.step_num[e] = step_num;
        envbits[tid] = bits;
    }
    __syncthreads();
    STAMP(4);

    // ---- phase 4: observations of re-initialised envs (:105)
    if (tid < nr && (envbits[el] & kFin)) {
        observe_row<A_T, O_T, false>(A, O, st + 5 * A * el, ob + 2 * S * el, tg + 2 * el, a,
                                     obs + tid * D, pr);
    }
    __syncthreads();
    STAMP(5);

    // ---- phase 5: stream the tile out
    tile_store(b.states + e0 * A * 5, st, nr * 5, tid, nthr);
    tile_store(b.obs + e0 * A * D, obs, nr * D, tid, nthr);
    if (norm)
        tile_store_norm(b.obs_norm + e0 * A * D, obs, nr * D, D, lds + tp.off_nm,
                        lds + tp.off_ns, tid, nthr);
    if (tid < 3 && b.counters) {
        const unsigned v = cnt[tid];
        if (v) b.counters[tid * args.slots + blockIdx.x] += v;
    }
    STAMP(6);
#if MARLNAV_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(7);
#endif
}

// ------------------------------------------------------------ observe kernel
template <int A_T, int O_T>
__global__ void __launch_bounds__(1024) observe_kernel(StepArgs args)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int A = A_T ? A_T : args.A;
    const int O = O_T ? O_T : args.O;
    const int S = args.S;
    const TilePlan tp = make_plan(args.E, A, O, S);
    const int E = tp.E, D = tp.D;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * E;
    const int ne = (int)((args.P - e0) < E ? (args.P - e0) : E);
    const int nr = ne * A;
    float *st = lds + tp.off_st;
    float *ob = lds + tp.off_ob;
    float *tg = lds + tp.off_tg;
    float *obs = lds + tp.off_obs;
    stage_spans<4>(Span{args.b.states + e0 * A * 5, st, nr * 5},
                   Span{args.b.obstacles + e0 * S * 2, ob, ne * S * 2},
                   Span{args.b.target + e0 * 2, tg, ne * 2}, tid, nthr);
    __syncthreads();
    if (tid < nr) {
        const int el = tid / A, a = tid - el * A;
        MarlnavParams pr{};
        pr.cap_distance = 0.1f;
        observe_row<A_T, O_T, false>(A, O, st + 5 * A * el, ob + 2 * S * el, tg + 2 * el, a,
                                     obs + tid * D, pr);
    }
    __syncthreads();
    tile_store(args.b.obs + e0 * A * D, obs, nr * D, tid, nthr);
}

// ----------------------------------------------------- native reinit kernel
__global__ void reinit_all_kernel(int64_t P, int A, int S, int64_t env_offset, uint64_t sidx,
                                  MarlnavParams pr, const float *__restrict__ formation,
                                  float *states, float *obstacles, float *target)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P) return;
    native_fresh_env(A, S, pr, formation, (uint64_t)(env_offset + e), sidx, states + e * A * 5,
                     obstacles + e * S * 2, target + 2 * e);
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
int pick_envs_per_tile(int A, int O, int S)
{
    int E = 64;
    while (E > 1 && (E * A > 1024 || make_plan(E, A, O, S).bytes > kLdsBudget)) E >>= 1;
    return E;
}

int validate(const MarlnavDims *d)
{
    if (!d) return fail(MARLNAV_EINVAL, "dims is NULL");
    if (d->num_parallel < 1) return fail(MARLNAV_EINVAL, "num_parallel=%lld < 1", (long long)d->num_parallel);
    if (d->num_agents < 2 || d->num_agents > kMaxAgents)
        return fail(MARLNAV_EINVAL, "num_agents=%d outside [2, %d]", d->num_agents, kMaxAgents);
    if (d->num_obstacles < 1 || d->num_obstacles > d->obstacle_stride)
        return fail(MARLNAV_EINVAL, "num_obstacles=%d outside [1, obstacle_stride=%d]",
                    d->num_obstacles, d->obstacle_stride);
    if (d->obstacle_stride > kMaxStride)
        return fail(MARLNAV_EINVAL, "obstacle_stride=%d > %d", d->obstacle_stride, kMaxStride);
    const int E = pick_envs_per_tile(d->num_agents, d->num_obstacles, d->obstacle_stride);
    if (make_plan(E, d->num_agents, d->num_obstacles, d->obstacle_stride).bytes > 64 * 1024)
        return fail(MARLNAV_EUNSUPPORTED, "tile does not fit LDS for A=%d O=%d S=%d",
                    d->num_agents, d->num_obstacles, d->obstacle_stride);
    return 0;
}

using StepFn = void (*)(StepArgs, MarlnavParams);
using ObsFn = void (*)(StepArgs);

struct KernelPair {
    int A, O;
    StepFn step;
    ObsFn obs;
};

const KernelPair kVariants[] = {
    {3, 3, step_kernel<3, 3>, observe_kernel<3, 3>},
    {3, 8, step_kernel<3, 8>, observe_kernel<3, 8>},
    {3, 1, step_kernel<3, 1>, observe_kernel<3, 1>},
    {2, 1, step_kernel<2, 1>, observe_kernel<2, 1>},
    {16, 32, step_kernel<16, 32>, observe_kernel<16, 32>},
};

KernelPair select_kernels(int A, int O)
{
    for (const KernelPair &k : kVariants)
        if (k.A == A && k.O == O) return k;
    return KernelPair{0, 0, step_kernel<0, 0>, observe_kernel<0, 0>};
}

int launch_check(const char *what)
{
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MARLNAV_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
    return 0;
}

StepArgs make_args(const MarlnavDims *d, int E)
{
    StepArgs a;
    memset(&a, 0, sizeof(a));
    a.P = d->num_parallel;
    a.env_offset = d->env_offset;
    a.E = E;
    a.A = d->num_agents;
    a.O = d->num_obstacles;
    a.S = d->obstacle_stride;
    a.slots = (d->num_parallel + E - 1) / E;
    return a;
}

}  // namespace

extern "C" {

int marlnav_abi_version(void) { return MARLNAV_ABI_VERSION; }

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
    const int E = pick_envs_per_tile(d->num_agents, d->num_obstacles, d->obstacle_stride);
    return (d->num_parallel + E - 1) / E;
}

int marlnav_step(const MarlnavDims *d, const MarlnavParams *pr, const MarlnavStepBuffers *b,
                 uint64_t step_idx, void *stream)
{
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
    const int A = d->num_agents, O = d->num_obstacles, S = d->obstacle_stride;
    const int E = pick_envs_per_tile(A, O, S);
    const TilePlan tp = make_plan(E, A, O, S);
    StepArgs args = make_args(d, E);
    args.b = *b;
    args.step_idx = step_idx;
    const KernelPair k = select_kernels(A, O);
    const dim3 grid((unsigned)args.slots), block((unsigned)tp.R);
    MarlnavParams prv = *pr;
    void *kargs[] = {&args, &prv};
    const hipError_t e = hipLaunchKernel(reinterpret_cast<const void *>(k.step), grid, block,
                                         kargs, (size_t)tp.bytes, (hipStream_t)stream);
    if (e != hipSuccess) return fail(MARLNAV_ELAUNCH, "marlnav_step: %s", hipGetErrorString(e));
    return launch_check("marlnav_step");
}

int marlnav_observe(const MarlnavDims *d, const float *states, const float *obstacles,
                    const float *target, float *obs, void *stream)
{
    if (int rc = validate(d)) return rc;
    if (!states || !obstacles || !target || !obs)
        return fail(MARLNAV_EINVAL, "a required observe buffer is NULL");
    const int A = d->num_agents, O = d->num_obstacles, S = d->obstacle_stride;
    const int E = pick_envs_per_tile(A, O, S);
    const TilePlan tp = make_plan(E, A, O, S);
    StepArgs args = make_args(d, E);
    args.b.states = const_cast<float *>(states);
    args.b.obstacles = const_cast<float *>(obstacles);
    args.b.target = const_cast<float *>(target);
    args.b.obs = obs;
    const KernelPair k = select_kernels(A, O);
    void *kargs[] = {&args};
    const hipError_t e = hipLaunchKernel(reinterpret_cast<const void *>(k.obs),
                                         dim3((unsigned)args.slots), dim3((unsigned)tp.R), kargs,
                                         (size_t)tp.bytes, (hipStream_t)stream);
    if (e != hipSuccess) return fail(MARLNAV_ELAUNCH, "marlnav_observe: %s", hipGetErrorString(e));
    return launch_check("marlnav_observe");
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
    return launch_check("marlnav_reinit_all");
}

int marlnav_counters_total(const MarlnavDims *d, const uint64_t *counters, uint64_t *out3,
                           void *stream)
{
    const int64_t slots = marlnav_counter_slots(d);
    if (slots < 0) return MARLNAV_EINVAL;
    if (!counters || !out3) return fail(MARLNAV_EINVAL, "counters/out3 is NULL");
    hipLaunchKernelGGL(counters_total_kernel, dim3(3), dim3(64), 0, (hipStream_t)stream,
                       counters, slots, out3);
    return launch_check("marlnav_counters_total");
}

}  // extern "C"
