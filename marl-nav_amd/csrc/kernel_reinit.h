// kernel_reinit.h - workgroup-spread re-initialisation and re-observation of finished envs (environment.py:76-90, 105), shared by the split and block kernels.
// Part of libmarlnav.so: included once, by marlnav_step.hip (one translation
// unit), inside its anonymous namespace.
#pragma once

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

// reobs_block for re-initialised envs that all equal the native fresh env
// in their agent rows and target (reinit_block found no `unclean` env): the
// target and agent-agent pairs come from the formation template `tpl`
// (marlnav_formation_obs: raw bearing, distance), only the agent-obstacle
// pairs are computed. Item (env, agent, obstacle j) also writes the template
// pairs m = j, j + O, ... < A of its agent row.
template <int A, int O, class Envs, class List>
__device__ __forceinline__ void reobs_block_tpl(const Envs &ev, const List &list, int nfin,
                                                float cap, const float2 *__restrict__ tpl,
                                                int tid, int nt)
{
    const int nw = nfin * A * O;
    for (int base = 0; base < nw; base += nt) {
        const int w = base + tid;
        const bool on = w < nw;
        const int wc = on ? w : 0;
        const int fe = wc / (A * O), rem = wc - fe * (A * O);
        const int ag = rem / O, j = rem - ag * O;
        const int c = list[fe];
        const float *s = ev.state(c) + 5 * ag;
        const float ox = s[0], oy = s[1], dx = s[2], dy = s[3];
        const float *pt = ev.obst(c) + 2 * j;
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
            o[2 + j] = ang;
            o[2 + O + j] = d;
            for (int m = j; m < A; m += O) {
                const float2 t = tpl[ag * A + m];
                const int sa = m == 0 ? 0 : 2 + 2 * O + (m - 1);
                const int sd = m == 0 ? 1 : 2 + 2 * O + (A - 1) + (m - 1);
                o[sa] = t.y < cap ? 0.0f : t.x;  // the cap (environment.py:172-177)
                o[sd] = t.y;
            }
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

// The block's fresh obstacle draws precomputed while its staging loads are in
// flight (env-block and few-obstacle split kernels): `pre` holds component k
// (0 x, 1 y) of obstacle j of env code c at pre[(2j + k) * E + c]
// (native_obst_draw, device_math.h).

// Re-initialisation of the finished envs (environment.py:76-90, the sampler
// call at :78) spread over the workgroup: one item per thread per pass - one
// float of a fresh candidate (reference RNG) or of the formation template,
// or one obstacle's Philox block (native; the same draws as
// native_fresh_env). Writes the LDS state and the global obstacles / target;
// the agent rows go out with the final stores.
// `unclean` (optional, native re-init): set to 1 when a finished env's
// blended agent coordinates or target differ from the formation's bits (a
// non-finite old value blends to NaN), i.e. when the formation template
// (reobs_block_tpl) does not describe the re-initialised env.
// E > 0 (native re-init): the fresh obstacles come from `pre` (E envs,
// native_obst_draw at stage time) instead of being drawn here.
template <int A, int O, int E = 0, class Envs, class List>
__device__ __forceinline__ void reinit_block(KArgsK *kl, const Envs &ev, const float *form,
                                             const List &list, int nfin, int tid, int nt,
                                             int *unclean = nullptr, const float *pre = nullptr)
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
                out_el(gob, e * O * 2 + j, v);
            } else {
                const int j = kk - 5 * A - 2 * O;
                float *d = ev.targ(c) + j;
                const float v = blend_in(*d, ft[2 * e + j]);
                *d = v;
                out_el(gtg, 2 * e + j, v);
            }
        }
        return;
    }
    constexpr int NI = 5 * A + 2 + O;
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
            const float v = blend_in(*d, form[kk]);
            *d = v;
            if (unclean && kk % 5 < 4 && __float_as_uint(v) != __float_as_uint(form[kk]))
                *unclean = 1;
        } else if (kk < 5 * A + 2) {
            const int j = kk - 5 * A;
            float *d = ev.targ(c) + j;
            const float v = blend_in(*d, form[kk]);
            *d = v;
            out_el(gtg, 2 * e + j, v);
            if (unclean && __float_as_uint(v) != __float_as_uint(form[kk])) *unclean = 1;
        } else {
            const int j = kk - 5 * A - 2;  // obstacle j
            float v[2];
            if constexpr (E > 0) {
                v[0] = pre[(2 * j) * E + c];
                v[1] = pre[(2 * j + 1) * E + c];
            } else {
                native_obst_draw(seed, sidx, (uint64_t)(eoff + e), j, rx, mx, ry, my, v);
            }
            float *o = ev.obst(c) + 2 * j;
            const int64_t g = e * O * 2 + 2 * j;
            o[0] = blend_in(o[0], v[0]);
            o[1] = blend_in(o[1], v[1]);
            out_el(gob, g, o[0]);
            out_el(gob, g + 1, o[1]);
        }
    }
}

// Native (non-noisy) re-init and re-observation of the finished envs in ONE
// pass over the workgroup: a fresh env's agent rows and target are the
// formation template and its obstacles are Philox draws (the same as
// native_fresh_env), so each observation item computes its own inputs
// instead of waiting for a re-init pass and a barrier. Items per finished
// env: A*(1+O+A-1) pairs (written into the packed rows), 5A+2 template
// floats and O Philox blocks, one per obstacle (written to the LDS state and
// the global obstacles/target).
//
// With two or more waves the items go by kind: the first half of the waves
// takes the pair items, the rest the template / obstacle items, so no wave
// runs both code paths one after the other (the pass is the tail of the
// block: issue-bound on the few waves that have items). A wave with no item
// left skips the pass. `tid` and `nt` are wave-aligned.
template <int A, int O>
struct NativeItems {
    static constexpr int NP = 1 + O + (A - 1);
    static constexpr int NPAIR = A * NP, NREST = 5 * A + 2 + O;
};


// pair item kk (< NPAIR) of finished env c; `on` false: computes, stores nothing.
// PRE: fresh obstacles from `pre` (E envs per block), else drawn here.
template <int A, int O, int E, class Envs>
__device__ __forceinline__ void native_pair_item(KArgsK *kl, const Envs &ev, const float *form,
                                                 const float *pre, int c, int kk, bool on, float cap)
{
    using IT = NativeItems<A, O>;
    const int ag = kk / IT::NP, p = kk - ag * IT::NP;
    uint32_t ux = 0u, uy = 0u;
    const bool cargs = (MARLNAV_AB & 8) != 0;  // timing only: no kernel-argument loads
    if (!E && p >= 1 && p <= O)  // obstacle p - 1: its Philox block
        native_block(cargs ? 5u : kl->p.seed, (uint32_t)(p - 1),
                     (uint64_t)((cargs ? 0 : kl->a.env_offset) + ev.env(c)),
                     cargs ? 7u : kl->a.step_idx, ux, uy);
    // inputs: the blend of the env's current value (LDS; other items may be
    // blending it in place meanwhile - blend_in is idempotent) with its fresh
    // value (template or Philox draw)
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
        const float *oo = ev.obst(c) + 2 * (p - 1);
        if constexpr (E > 0) {
            px = blend_in(oo[0], pre[(2 * (p - 1)) * E + c]);
            py = blend_in(oo[1], pre[(2 * (p - 1) + 1) * E + c]);
        } else {
            const float rx = cargs ? 1000.f : kl->p.obs_range_x, mx = cargs ? 0.f : kl->p.obs_mean_x;
            const float ry = cargs ? 1000.f : kl->p.obs_range_y, my = cargs ? 0.f : kl->p.obs_mean_y;
            px = blend_in(oo[0], rx * (native_u24(ux) - 0.5f) + mx);
            py = blend_in(oo[1], ry * (native_u24(uy) - 0.5f) + my);
        }
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
    if (MARLNAV_AB & 16) {  // timing only: no pair math
        d = px + ox + dx;
        ang = py + oy + dy;
    } else if (__ballot(on && !cok) == 0ull) {
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

// template / obstacle item k2 (< NREST) of finished env c (PRE as above)
// TailOut (the env-block kernel's kTailOut): the global obstacles / target of
// the block's envs from the caller's SGPR pointers (instead of kernarg
// loads) and, with `wt`, written through with offsets from the block's
// first env.
struct TailOut {
    float *gob, *gtg;
    int64_t e0;
    bool wt;
};

template <int O>
__device__ __forceinline__ void tail_out(const TailOut *to, KArgsK *kl, bool obst, int64_t idx,
                                         float v)
{
    if (to == nullptr) {
        out_el(obst ? kl->a.b.obstacles : kl->a.b.target, idx, v);
    } else if (kWtOut && to->wt) {
        const int64_t base = obst ? to->e0 * O * 2 : to->e0 * 2;
        const uint32_t span = obst ? 64u * O * 2 * 4 : 64u * 2 * 4;
        wt_st(out_buf((obst ? to->gob : to->gtg) + base, span), (uint32_t)(idx - base) * 4u, v);
    } else {
        out_el(obst ? to->gob : to->gtg, idx, v);
    }
}

template <int A, int O, int E, class Envs>
__device__ __forceinline__ void native_rest_item(KArgsK *kl, const Envs &ev, const float *form,
                                                 const float *pre, int c, int k2,
                                                 const TailOut *to = nullptr)
{
    const int64_t e = ev.env(c);
    if (k2 < 5 * A) {
        float *d = ev.state(c) + k2;
        *d = blend_in(*d, form[k2]);
    } else if (k2 < 5 * A + 2) {
        const int j = k2 - 5 * A;
        float *d = ev.targ(c) + j;
        const float v = blend_in(*d, form[k2]);
        *d = v;
        tail_out<O>(to, kl, false, 2 * e + j, v);
    } else {
        const int j = k2 - (5 * A + 2);  // obstacle j
        float v[2];
        if constexpr (E > 0) {
            v[0] = pre[(2 * j) * E + c];
            v[1] = pre[(2 * j + 1) * E + c];
        } else {
            native_obst_draw(kl->p.seed, kl->a.step_idx, (uint64_t)(kl->a.env_offset + e), j,
                             kl->p.obs_range_x, kl->p.obs_mean_x, kl->p.obs_range_y,
                             kl->p.obs_mean_y, v);
        }
        float *o = ev.obst(c) + 2 * j;
        const int64_t g = e * O * 2 + 2 * j;
        o[0] = blend_in(o[0], v[0]);
        o[1] = blend_in(o[1], v[1]);
        tail_out<O>(to, kl, true, g, o[0]);
        tail_out<O>(to, kl, true, g + 1, o[1]);
    }
}

// Native re-init and re-observation of the finished envs of many-obstacle
// shapes (pair-split kernel, kSplitTpl) in ONE pass over the workgroup, with
// the formation `form` and its observation template `tpl`
// (marlnav_formation_obs) staged in LDS with the tile. Per finished env and
// thread: the Philox block of one obstacle j (the draws native_fresh_env
// makes; thread j < O also blends obstacle j into LDS and the global
// obstacles), that obstacle's pairs with agents tid / O, tid / O + nt / O, ...
// (the agents' blends computed by the item), one template pair (target or
// other agent: copied, with the distance cap) and at most one blend of the
// state or target (LDS; the global target). The items run concurrently:
// blend_in is idempotent, so an item that reads a value another item already
// blended gets the same bits. The template pairs hold only when every agent
// coordinate and the target blend to the formation's bits; a blend item that
// finds otherwise (a non-finite old value) sets `unclean`, and the caller then
// recomputes every pair (reobs_block) after the barrier that ends this pass.
// NT threads (all of the workgroup's), a multiple of O: a thread's pairs are
// compile-time unrolled, so their chains interleave.
template <int A, int O, int NT, class Envs, class List>
__device__ __forceinline__ void reinit_reobs_tpl(KArgsK *kl, const Envs &ev, const float *form,
                                                 const float2 *__restrict__ tpl, const List &list,
                                                 int nfin, float cap, int tid, int *unclean)
{
    static_assert(NT % O == 0, "whole obstacle columns per pass");
    constexpr int agd = NT / O;
    float *gob = kl->a.b.obstacles;
    float *gtg = kl->a.b.target;
    const uint64_t seed = kl->p.seed, sidx = kl->a.step_idx;
    const int64_t eoff = kl->a.env_offset;
    const float rx = kl->p.obs_range_x, mx = kl->p.obs_mean_x;
    const float ry = kl->p.obs_range_y, my = kl->p.obs_mean_y;
    const int j = tid % O, ag0 = tid / O;
    if constexpr (MARLNAV_TPL_LOADS_FIRST && A * A <= NT && 5 * A + 2 <= NT) {
        // (A/B) every LDS read of the pass first, then the Philox block and
        // the pair math, then every write: one LDS round trip in front of
        // the chain instead of one per step
        constexpr int KA = (A + agd - 1) / agd;
        for (int fe = 0; fe < nfin; ++fe) {
            const int c = list[fe];
            const int64_t e = ev.env(c);
            const bool has_t = tid < A * A;
            const float2 tv = tpl[has_t ? tid : 0];
            const int k2 = tid;
            const bool has_b = k2 < 5 * A + 2;
            const bool btg = k2 >= 5 * A;
            float *bd = btg ? ev.targ(c) + (k2 - 5 * A) : ev.state(c) + (has_b ? k2 : 0);
            const float bold = *bd, bform = form[has_b ? k2 : 0];
            const float *oo = ev.obst(c) + 2 * j;
            const float oox = oo[0], ooy = oo[1];
            float so[KA][4], sf[KA][4];
#pragma unroll
            for (int k = 0; k < KA; ++k) {
                const int ag = ag0 + k * agd;
                const int agc = ag < A ? ag : 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    so[k][q] = ev.state(c)[5 * agc + q];
                    sf[k][q] = form[5 * agc + q];
                }
            }
            float v[2];
            native_obst_draw(seed, sidx, (uint64_t)(eoff + e), j, rx, mx, ry, my, v);
            const float px = blend_in(oox, v[0]);
            const float py = blend_in(ooy, v[1]);
            float dd[KA], aa[KA];
#pragma unroll
            for (int k = 0; k < KA; ++k) {
                const bool on = ag0 + k * agd < A;
                const float ox = blend_in(so[k][0], sf[k][0]), oy = blend_in(so[k][1], sf[k][1]);
                const float dx = blend_in(so[k][2], sf[k][2]), dy = blend_in(so[k][3], sf[k][3]);
                const bool cok = coord_ok(ox) && coord_ok(oy) && coord_ok(px) && coord_ok(py);
                bool unused = true;
                if (__ballot(on && !cok) == 0ull) {
                    dd[k] = pair_dist<true>(ox, oy, px, py, unused);
                    aa[k] = pair_angle<true>(ox, oy, px, py, dx, dy, dd[k], cap, unused);
                } else {
                    dd[k] = pair_dist<false>(ox, oy, px, py, unused);
                    aa[k] = pair_angle<false>(ox, oy, px, py, dx, dy, dd[k], cap, unused);
                }
            }
            // writes: template pair, blend, the pairs, the obstacle
            if (has_t) {
                const int ag = tid / A, m = tid - ag * A;
                const int sa = m == 0 ? 0 : 2 + 2 * O + (m - 1);
                const int sd = m == 0 ? 1 : 2 + 2 * O + (A - 1) + (m - 1);
                float *o = ev.row(c, ag);
                o[sa] = tv.y < cap ? 0.0f : tv.x;  // the cap (environment.py:172-177)
                o[sd] = tv.y;
            }
            if (has_b) {
                const float vb = blend_in(bold, bform);
                *bd = vb;
                if (btg) out_el(gtg, 2 * e + (k2 - 5 * A), vb);
                if ((btg || k2 % 5 < 4) && __float_as_uint(vb) != __float_as_uint(bform)) *unclean = 1;
            }
#pragma unroll
            for (int k = 0; k < KA; ++k) {
                const int ag = ag0 + k * agd;
                if (ag < A) {
                    float *o = ev.row(c, ag);
                    o[2 + j] = aa[k];
                    o[2 + O + j] = dd[k];
                }
            }
            if (ag0 == 0) {
                float *ow = ev.obst(c) + 2 * j;
                ow[0] = px;
                ow[1] = py;
                out_el(gob, e * O * 2 + 2 * j, px);
                out_el(gob, e * O * 2 + 2 * j + 1, py);
            }
        }
        return;
    }
    for (int fe = 0; fe < nfin; ++fe) {
        const int c = list[fe];
        const int64_t e = ev.env(c);
        // (the template copies and blends first: their LDS round trips run
        // under the Philox chain that follows)
        // template pairs: m = 0 the target, m >= 1 other agent m - 1
#pragma unroll
        for (int p = tid; p < A * A; p += NT) {
            const int ag = p / A, m = p - ag * A;
            const float2 t = tpl[p];
            const int sa = m == 0 ? 0 : 2 + 2 * O + (m - 1);
            const int sd = m == 0 ? 1 : 2 + 2 * O + (A - 1) + (m - 1);
            float *o = ev.row(c, ag);
            o[sa] = t.y < cap ? 0.0f : t.x;  // the cap (environment.py:172-177)
            o[sd] = t.y;
        }
        // blends of the state and target (environment.py:76-90)
        for (int k2 = tid; k2 < 5 * A + 2; k2 += NT) {
            const bool tg = k2 >= 5 * A;
            float *d = tg ? ev.targ(c) + (k2 - 5 * A) : ev.state(c) + k2;
            const float vb = blend_in(*d, form[k2]);
            *d = vb;
            if (tg) out_el(gtg, 2 * e + (k2 - 5 * A), vb);
            if ((tg || k2 % 5 < 4) && __float_as_uint(vb) != __float_as_uint(form[k2]))
                *unclean = 1;
        }
        // obstacle j: its Philox block and blend
        float v[2];
        native_obst_draw(seed, sidx, (uint64_t)(eoff + e), j, rx, mx, ry, my, v);
        const float *oo = ev.obst(c) + 2 * j;
        const float px = blend_in(oo[0], v[0]);
        const float py = blend_in(oo[1], v[1]);
        // its pairs with agents ag0, ag0 + agd, ... (per wave and agent: the
        // short sqrt / division sequences when every coordinate passes
        // coord_ok, IEEE otherwise)
#pragma unroll
        for (int k = 0; k * agd < A; ++k) {
            const int ag = ag0 + k * agd;
            const bool on = ag < A;
            const float *s = form + 5 * (on ? ag : 0), *so = ev.state(c) + 5 * (on ? ag : 0);
            const float ox = blend_in(so[0], s[0]), oy = blend_in(so[1], s[1]);
            const float dx = blend_in(so[2], s[2]), dy = blend_in(so[3], s[3]);
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
                o[2 + j] = ang;
                o[2 + O + j] = d;
            }
        }
        if (ag0 == 0) {  // (after this thread's own reads of the old obstacle)
            float *ow = ev.obst(c) + 2 * j;
            ow[0] = px;
            ow[1] = py;
            out_el(gob, e * O * 2 + 2 * j, px);
            out_el(gob, e * O * 2 + 2 * j + 1, py);
        }
    }
}

// The finished envs of a block as a wave-uniform ballot mask (env code = bit
// position; the env-block kernel): entry fe is the fe-th set bit, found by
// scalar bit scans over the few entries one pass of items touches - no LDS
// list to write, wait for and read back.
struct MaskList {
    uint64_t fm;
};

// env code of entry fe, for the entries [lo, hi] of one pass (wave-uniform)
template <class List>
__device__ __forceinline__ int list_code(const List &l, int fe, int, int)
{
    return l[fe];
}

__device__ __forceinline__ int list_code(const MaskList &l, int fe, int lo, int hi)
{
    uint64_t m = l.fm;
    for (int f = 0; f < lo; ++f) m &= m - 1;
    int c = 0;
    for (int f = lo; f <= hi; ++f) {
        const int pos = (int)__builtin_ctzll(m);
        c = fe == f ? pos : c;
        m &= m - 1;
    }
    return c;
}

// E > 0: fresh obstacles precomputed in `pre` (E envs, native_obst_draw)
template <int A, int O, int E = 0, class Envs, class List>
__device__ __forceinline__ void reinit_reobs_native(KArgsK *kl, const Envs &ev, const float *form,
                                                    const List &list, int nfin, float cap, int tid,
                                                    int nt, const float *pre = nullptr,
                                                    const TailOut *to = nullptr)
{
    using IT = NativeItems<A, O>;
    constexpr int NI = IT::NPAIR + IT::NREST;
    // (tid and nt are wave-aligned: the wave index is uniform)
    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6), nwv = nt >> 6;
    if (nwv >= 2) {
        const int pw = nwv >> 1;  // waves [0, pw): pair items; [pw, nwv): the rest
        if (wv < pw) {
            if (MARLNAV_AB & (1 << 18)) return;  // (timing only: no pair items)
            const int n = nfin * IT::NPAIR;
            for (int base = 64 * wv; base < n; base += 64 * pw) {
                const int i = base + lane;
                const bool on = i < n;
                const int ic = on ? i : 0;
                const int fe = ic / IT::NPAIR;
                const int lo = base / IT::NPAIR, hi = min((base + 63) / IT::NPAIR, nfin - 1);
                native_pair_item<A, O, E>(kl, ev, form, pre, list_code(list, fe, lo, hi),
                                          ic - fe * IT::NPAIR, on, cap);
            }
        } else {
            if (MARLNAV_AB & (1 << 17)) return;  // (timing only: no template / obstacle items)
            const int n = nfin * IT::NREST;
            for (int base = 64 * (wv - pw); base < n; base += 64 * (nwv - pw)) {
                const int i = base + lane;
                const int lo = base / IT::NREST, hi = min((base + 63) / IT::NREST, nfin - 1);
                const int fe = (i < n ? i : 0) / IT::NREST;
                const int c = list_code(list, fe, lo, hi);
                if (i < n) native_rest_item<A, O, E>(kl, ev, form, pre, c, i - fe * IT::NREST, to);
            }
        }
        return;
    }
    const int n = nfin * NI;
    for (int base = 64 * wv; base < n; base += nt) {
        const int i = base + lane;
        const bool on = i < n;
        const int ic = on ? i : 0;
        const int fe = ic / NI, kk = ic - fe * NI;
        const int c = list_code(list, fe, base / NI, min((base + 63) / NI, nfin - 1));
        if (kk < IT::NPAIR)
            native_pair_item<A, O, E>(kl, ev, form, pre, c, kk, on, cap);
        else if (on)
            native_rest_item<A, O, E>(kl, ev, form, pre, c, kk - IT::NPAIR, to);
    }
}
