// kernel_block.h - env-block kernel (one workgroup of A waves per 64 envs: the A3 headline path).
// Part of libmarlnav.so: included once, by marlnav_step.hip (one translation
// unit), inside its anonymous namespace.
#pragma once

// ------------------------------------------------------- env-block kernel
// One workgroup of A waves per block of E = 64 consecutive envs: lane l of
// wave w owns agent w of env l. Every lane holds a row (wave tiles of whole
// envs - the round-1 tile family - left 64 - 3*20 = 4 lanes idle at A3), the
// agent index is wave-uniform, and the per-env phase runs once per block on
// wave 0 with all 64 lanes busy instead of on 20 of 64 lanes in every wave.
// Grid shape: at 65536 envs x 3 agents, 1024 blocks of 3 waves = 3 waves on
// every SIMD, where 64/3-env wave tiles give 3277 waves and a fifth of the
// SIMDs a fourth wave (measured by scripts/kstamps.py: those SIMDs set the
// kernel's end).
// Rows are exchanged through LDS between block barriers (5 per step); the
// packed observation rows are assembled in LDS and streamed out as one
// contiguous span (a store instruction covers 1 KiB, 8 cache lines, where
// register-row stores at a 48-byte lane stride touch 24).
// LPR lanes per agent row (1, 2 or 4): E = 64 / LPR envs per block. LPR > 1
// splits each row's pairs over LPR neighbouring lanes, for grids too small to
// give every SIMD three waves at one lane per row (16384 envs: 256 blocks of
// 64 leave a quarter of the SIMDs idle and each wave alone on its SIMD; at
// LPR 4, 1024 blocks of 16 give every SIMD three waves, each with a third of
// the pairs per lane).
template <int A, int O, int LPR = 1, bool HELP = false>
struct BlockPlan {
    static_assert(LPR == 1 || LPR == 2 || LPR == 4, "lanes per row: 1, 2 or 4");
    static_assert(!HELP || LPR == 1, "the helper wave serves one-lane-per-row blocks");
    static constexpr int E = 64 / LPR, R = E * A, D = 2 + 2 * O + 2 * (A - 1);
    static constexpr int NT = 64 * A;                      // threads per block
    static constexpr int ST = 0;                           // (R, 5)
    static constexpr int ACTW = (ST + R * 5 + 3) & ~3;     // (A, 2, E) actions, per wave
    static constexpr int OB = (ACTW + 2 * R + 3) & ~3;     // (E, O, 2)
    static constexpr int TG = (OB + E * O * 2 + 3) & ~3;   // (E, 2)
    static constexpr int SN = (TG + E * 2 + 3) & ~3;       // (E,)
    static constexpr int TM = (SN + E + 3) & ~3;           // (E,) bytes
    static constexpr int FORM = (TM + E / 4 + 3) & ~3;     // 5A + 2 (native re-init)
    static constexpr int RED = (FORM + 5 * A + 2 + 3) & ~3;  // (R, 4) reward terms
    static constexpr int OBS = RED + 4 * R;                // (R, D) packed rows
    static constexpr int LIST = (OBS + R * D + 3) & ~3;    // (E,) finished envs
    static constexpr int FLG = LIST + E;                   // [0] nfin, [1 + w] wave w coords bad
    static constexpr int FRESH = (FLG + 1 + A + 3) & ~3;   // (2O, E) fresh obstacle draws
    static constexpr int PT = FRESH + 2 * O * E;           // (A, E) float2 agent-pair terms (A3)
    // (HELP) the fresh env's agent-obstacle pairs, (E, A, 2O): bearing then distance
    static constexpr int FR = PT + (A == 3 ? 2 * A * E : 0);
    static constexpr int FLOATS = FR + (HELP ? 2 * O * A * E : 0);
    static_assert(A >= 2 && A <= 16, "one wave per agent");
};

// Copy NB bytes of the block's span k into LDS by LDS-DMA from the wave
// k % A (spans spread over the block's waves).
template <int NB, int AUX = 0>
__device__ __forceinline__ void block_glds(int k, int A, int w, const void *src, float *dst,
                                           unsigned lane)
{
    if (k % A == w) glds_span<NB, AUX>(src, dst, lane);
}

// LDS-DMA instructions glds_span<NB> issues (one per KiB, one for the tail)
__host__ __device__ constexpr int glds_count(int NB)
{
    return (NB / 16 + 63) / 64 + ((NB % 16) / 4 > 0 ? 1 : 0);
}

// The staging spans of a full block, in issue order: span id k (issued by
// wave k % A) and its byte count. The issue sites and the per-wave vmcnt
// that lets each wave use its own actions early both read this one table.
template <int A, int O, int LPR = 1>
struct BlockSpans {
    using BP = BlockPlan<A, O, LPR>;
    static constexpr int N = 6;
    // states, obstacles, target, step_num, terminates (step only), formation
    // (native re-init only)
    static constexpr int K[N] = {0, 1, 4, 2, 5, 7};
    static constexpr int NB[N] = {BP::R * 20, BP::E * O * 8, BP::E * 8, BP::E * 4, BP::E,
                                  (5 * A + 2) * 4};
    // LDS-DMA instructions wave w issues after its two action loads (the
    // formation span counted only when `formation`)
    static constexpr int after_actions(int w, bool formation)
    {
        int n = 0;
        for (int i = 0; i < N; ++i)
            if (K[i] % A == w && (i != N - 1 || formation)) n += glds_count(NB[i]);
        return n;
    }
};

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
                                            int n, int tid, int nt, bool wt)
{
    const int n4 = n >> 2;
    if (kWtOut && wt) {
        const OutBuf ob = out_buf(dst, (uint32_t)n * 4u);
        for (int i = tid; i < n4; i += nt)
            wt_st4(ob, 16u * i, reinterpret_cast<const float4 *>(src)[i]);
        for (int i = (n4 << 2) + tid; i < n; i += nt) wt_st(ob, 4u * i, src[i]);
        return;
    }
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
                                             int tid, bool wt)
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
    if (kWtOut && wt) {
        const OutBuf o1 = out_buf(d1, N1 * 4), o2 = out_buf(d2, N2 * 4);
#pragma unroll
        for (int k = 0; k < K1; ++k)
            if ((k + 1) * NT <= Q1 || tid + k * NT < Q1) wt_st4(o1, 16u * (tid + k * NT), v1[k]);
#pragma unroll
        for (int k = 0; k < K2; ++k)
            if ((k + 1) * NT <= Q2 || tid + k * NT < Q2) wt_st4(o2, 16u * (tid + k * NT), v2[k]);
        return;
    }
#pragma unroll
    for (int k = 0; k < K1; ++k)
        if ((k + 1) * NT <= Q1 || tid + k * NT < Q1) out_st4<kNtRows>(d1 + 4 * (tid + k * NT), v1[k]);
#pragma unroll
    for (int k = 0; k < K2; ++k)
        if ((k + 1) * NT <= Q2 || tid + k * NT < Q2) out_st4<kNtRows>(d2 + 4 * (tid + k * NT), v2[k]);
}


// LDS write of the first N floats of a register row to a row of stride D
// floats: the widest vector the row base's alignment allows (the block's rows
// start 16-byte aligned, so row r sits at 4*D*r bytes)
template <int N, int D>
__device__ __forceinline__ void lds_row_part_write(float *dst, const float *row)
{
    if constexpr (N % 4 == 0 && D % 4 == 0) {
#pragma unroll
        for (int k = 0; k < N; k += 4)
            *reinterpret_cast<float4 *>(dst + k) = make_float4(row[k], row[k + 1], row[k + 2], row[k + 3]);
    } else if constexpr (N % 2 == 0 && D % 2 == 0) {
#pragma unroll
        for (int k = 0; k < N; k += 2)
            *reinterpret_cast<float2 *>(dst + k) = make_float2(row[k], row[k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < N; ++k) dst[k] = row[k];
    }
}

// The observation phase of a FAST block at A = 3 with agent-pair symmetry
// (environment.py:139-180, 184-269). The three agents of an env have three
// unordered pairs; wave w takes pair (w, k = w + 1 mod 3) for its 64 envs and
// computes once what both directions share: the distance (the squares of
// +-dx are equal, so sqrtf(fmaf(dy,dy,dx*dx)) is the same bits both ways),
// the normalised difference (div2_fast is odd in the numerator and maps +-0
// to +0, so the reverse direction's quotient is exactly 0 - nx: no second
// division), the bond term and the risk / collision / band flags; then the
// two bearings (each from its own heading) go straight into both rows in LDS.
// Each wave then observes its own row's target and obstacles. After one
// block barrier the row's reward reads its two pairs' terms back (bond terms
// summed in torch's order over the others in index order).
// Every value equals what observe_row_own computes per direction; only the
// shared work is done once (per wave: one distance, one division, one bond
// term instead of two of each).
// EARLY (native, non-noisy re-init with the fresh obstacles drawn at stage
// time): the finished envs are known right after the block barrier - every
// collision flag of the env is in the pair terms then - so each wave
// re-initialises and re-observes its own agent's rows of the finished envs
// there (kernel_reinit.h native_pair_item / native_rest_item: the same items
// and values as reinit_reobs_native), before the observation barrier,
// instead of waves 1..A-1 doing all of it after that barrier while wave 0
// runs the per-env phase: the per-env phase then no longer waits for it.
struct EarlyReinit {
    KArgsK *kl;
    const float *form, *pre, *sn;
    const uint8_t *tm;
    float *ob, *tg;
    int64_t e0;
    int ne;
};

template <int A, int O, bool TERMS, bool REFC, bool EARLY = false>
__device__ __forceinline__ void block_observe_sym(float *__restrict__ st,
                                                  const float *__restrict__ obe,
                                                  const float *__restrict__ tge, int l, int w,
                                                  float ox, float oy, float dirx, float diry,
                                                  float *obs_rows, float2 *pt, float4 *red,
                                                  const MarlnavParams &pr,
                                                  const EarlyReinit &er = EarlyReinit{})
{
    static_assert(A == 3, "one unordered agent pair per wave");
    constexpr int E = BlockPlan<A, O>::E, D = BlockPlan<A, O>::D, NO = 2 + 2 * O;
    bool ok = true;  // (FAST block: every guard holds)
    const float cap = pr.cap_distance;
    // ---- the wave's agent pair (w, k)
    const int k = w == A - 1 ? 0 : w + 1;
    float pair_bt = 0.0f;
    unsigned pair_fl = 0u;  // bit0 agent risk, 1 agent collision, 2 in band; 3: row w's obstacle collision
    {
        const float *sk = st + 5 * (A * l + k);
        const float kx = sk[0], ky = sk[1], kdx = sk[2], kdy = sk[3];
        const float ddx = kx - ox, ddy = ky - oy;
        const float d = sqrt_fast(__builtin_fmaf(ddy, ddy, ddx * ddx), ok);
        const float den = __builtin_amdgcn_fmed3f(d, 1e-12f, __builtin_inff());
        float nx, ny;
        div2_fast(ddx, ddy, den, &nx, &ny, ok);
        const float a_wk = bearing_of<true>(nx, ny, dirx, diry, d, cap);
        const float a_kw = bearing_of<true>(0.0f - nx, 0.0f - ny, kdx, kdy, d, cap);
        // other k in row w at index k - (k > w); other w in row k at w - (w > k)
        const int jw = k - (k > w ? 1 : 0), jk = w - (w > k ? 1 : 0);
        float *rw = obs_rows + (A * l + w) * D + NO, *rk = obs_rows + (A * l + k) * D + NO;
        rw[jw] = a_wk;
        rw[(A - 1) + jw] = d;
        rk[jk] = a_kw;
        rk[(A - 1) + jk] = d;
        if (TERMS) {
            pair_bt = (pr.flags & kTermsFastFlag) ? bond_term<true, REFC>(d, pr, ok)
                                                  : bond_term<false>(d, pr, ok);
            pair_fl = (d < pr.ag_risk_dist ? 1u : 0u) | (d < pr.ag_coll_dist ? 2u : 0u) |
                      ((pr.agents_min_d < d && d < pr.agents_max_d) ? 4u : 0u);
        }
    }
    // ---- own row: target and obstacles
    float rowv[NO];
    const float td = pair_dist<true>(ox, oy, tge[0], tge[1], ok);
    const float ta = pair_angle<true>(ox, oy, tge[0], tge[1], dirx, diry, td, cap, ok);
    rowv[0] = ta;
    rowv[1] = td;
    bool ob_risk = false, ob_col = false;
#pragma unroll
    for (int j = 0; j < O; ++j) {
        const float px = obe[2 * j], py = obe[2 * j + 1];
        const float d = pair_dist<true>(ox, oy, px, py, ok);
        rowv[2 + j] = pair_angle<true>(ox, oy, px, py, dirx, diry, d, cap, ok);
        rowv[2 + O + j] = d;
        if (TERMS) {
            ob_risk |= d < pr.ob_risk_dist;
            ob_col |= d < pr.ob_coll_dist;
        }
    }
    lds_row_part_write<NO, D>(obs_rows + (A * l + w) * D, rowv);
    if (TERMS) {
        pt[w * E + l] = make_float2(pair_bt, __uint_as_float(pair_fl | (ob_col ? 8u : 0u)));
        __syncthreads();  // every pair's terms in LDS
        // the others of row w in index order, and the wave that owns each pair
        const int o0 = w == 0 ? 1 : 0, o1 = w == 2 ? 1 : 2;
        const int p0 = o0 == k ? w : o0, p1 = o1 == k ? w : o1;
        const float2 t0 = pt[p0 * E + l], t1 = pt[p1 * E + l];
        const unsigned f0 = __float_as_uint(t0.y), f1 = __float_as_uint(t1.y);
        float bt[A - 1] = {t0.x, t1.x};
        const float bond = torch_row_sum_r<A - 1>(bt, [](float x) { return x; });
        float band = 0.0f;
        band += (f0 & 4u) ? 1.0f : 0.0f;
        band += (f1 & 4u) ? 1.0f : 0.0f;
        const RowOut ro = row_reward<A, true, REFC>(ta, td, ob_risk || ((f0 | f1) & 1u) != 0,
                                                    ob_col || ((f0 | f1) & 2u) != 0, band, bond,
                                                    pr, ok);
        red[A * l + w] = make_float4(ro.r_miss, ro.r_hit, __uint_as_float(ro.flags), 0.0f);
        if constexpr (EARLY) {
            // finished (environment.py:96-104, 213-214): truncated, reached
            // the target last step, or any collision of the env's rows - every
            // agent pair's collision bit and every row's obstacle bit
            const int p2 = 3 - p0 - p1;  // the pair without agent w
            const unsigned f2 = __float_as_uint(pt[p2 * E + l].y);
            const unsigned fo = f0 | f1 | f2;
            const bool fin = l < er.ne && (er.sn[l] + 1.0f > pr.trunc_after || er.tm[l] != 0 ||
                                           (fo & 10u) != 0u);
            const uint64_t fm = __ballot(fin);  // (the same set in every wave)
            if (fm) {
                if (MARLNAV_TAIL_PRIO) __builtin_amdgcn_s_setprio(MARLNAV_TAIL_PRIO);  // (A/B)
                // wave w: agent w's rows of the finished envs - its NP pair
                // items and its 5 state floats; wave 0 also the target and the
                // obstacle blocks (LDS and global)
                using IT = NativeItems<A, O>;
                const BlockEnvs<A, O, D> ev{st, const_cast<float *>(er.ob), er.tg, obs_rows, er.e0};
                const int nfin = (int)__popcll(fm);
                const int ipw = IT::NP + 5 + (w == 0 ? 2 + IT::NB : 0);
                const int lane = (int)(threadIdx.x & 63);
                for (int base = 0; base < nfin * ipw; base += 64) {
                    const int i = base + lane;
                    const bool on = i < nfin * ipw;
                    const int ic = on ? i : 0;
                    const int fe = ic / ipw, rem = ic - fe * ipw;
                    const int lo = base / ipw, hi = min((base + 63) / ipw, nfin - 1);
                    const int c = list_code(MaskList{fm}, fe, lo, hi);
                    if (rem < IT::NP) {  // (every lane of the wave: the pair math's ballot)
                        native_pair_item<A, O, E>(er.kl, ev, er.form, er.pre, c, w * IT::NP + rem,
                                                  on, pr.cap_distance);
                    } else if (on) {
                        const int r2 = rem - IT::NP;
                        native_rest_item<A, O, E>(er.kl, ev, er.form, er.pre, c,
                                                  r2 < 5 ? 5 * w + r2 : 5 * A + (r2 - 5));
                    }
                }
            }
        }
    }
}

// Lane (row base + K) of an LPR-lane row group (LPR 2 or 4; groups are
// aligned within quads), read by every lane of the group: one DPP quad_perm.
template <int LPR, int K>
__device__ __forceinline__ float row_lane(float v)
{
    static_assert(LPR == 2 || LPR == 4, "row groups inside a quad");
    constexpr int q0 = (0 & ~(LPR - 1)) + K, q1 = (1 & ~(LPR - 1)) + K;
    constexpr int q2 = (2 & ~(LPR - 1)) + K, q3 = (3 & ~(LPR - 1)) + K;
    constexpr int ctrl = q0 | (q1 << 2) | (q2 << 4) | (q3 << 6);
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xf, 0xf, false));
}

template <int LPR, int K>
__device__ __forceinline__ unsigned row_lane_u(unsigned v)
{
    return __float_as_uint(row_lane<LPR, K>(__uint_as_float(v)));
}

// observations() of agent row `w` of one env (environment.py:139-180) with
// the row's NP = 1 + O + (A - 1) pairs split over LPR lanes: lane `sub` takes
// pairs sub, sub + LPR, ... (pair 0 the target, 1..O the obstacles, then the
// other agents in index order), writes their bearings and distances into the
// LDS row, and the row's reward terms (:184-269) are gathered onto lane
// sub = 0 through DPP (flags ORed, band counts added - whole numbers, so in
// any order - and the bond terms read back in the others' index order for
// torch's sum). Lane 0's RowOut is the row's; every value is the one
// observe_row_own computes.
template <int A, int O, int LPR, bool TERMS, bool FAST, bool REFC>
__device__ __forceinline__ RowOut observe_row_lpr(const float *__restrict__ sts,
                                                  const float *__restrict__ obe,
                                                  const float *__restrict__ tge, int w, int sub,
                                                  float ox, float oy, float dirx, float diry,
                                                  float *row, const MarlnavParams &pr)
{
    constexpr int NP = 1 + O + (A - 1), T = (NP + LPR - 1) / LPR;
    bool ok = true;  // (FAST: the block passed the coordinate check)
    const float cap = pr.cap_distance;
    const bool bt_fast = FAST && (pr.flags & kTermsFastFlag);
    float ta = 0.0f, td = 0.0f, band = 0.0f;
    unsigned fl = 0u;  // bit0 obstacle risk, 1 obstacle collision, 2 agent risk, 3 agent collision
    float bt[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int p = sub + LPR * t;
        bt[t] = 0.0f;
        if ((t + 1) * LPR <= NP || p < NP) {
            const bool is_tg = p == 0, is_ob = p >= 1 && p <= O;
            const int kx = p - O - 1;  // other agent index (p > O)
            const int m = kx + (kx >= w ? 1 : 0);
            const float *q = is_tg ? tge : (is_ob ? obe + 2 * (p - 1) : sts + 5 * m);
            const float px = q[0], py = q[1];
            const float d = pair_dist<FAST>(ox, oy, px, py, ok);
            const float ang = pair_angle<FAST>(ox, oy, px, py, dirx, diry, d, cap, ok);
            const int sa = is_tg ? 0 : (is_ob ? 1 + p : 2 + 2 * O + kx);
            const int sd = is_tg ? 1 : (is_ob ? 1 + O + p : 2 + 2 * O + (A - 1) + kx);
            row[sa] = ang;
            row[sd] = d;
            if (TERMS) {
                if (t == 0) {  // (pair 0 is lane 0's first)
                    ta = ang;
                    td = d;
                }
                fl |= is_ob ? ((d < pr.ob_risk_dist ? 1u : 0u) | (d < pr.ob_coll_dist ? 2u : 0u)) : 0u;
                const bool is_ag = p > O;
                fl |= is_ag ? ((d < pr.ag_risk_dist ? 4u : 0u) | (d < pr.ag_coll_dist ? 8u : 0u)) : 0u;
                band += (is_ag && pr.agents_min_d < d && d < pr.agents_max_d) ? 1.0f : 0.0f;
                bt[t] = bt_fast ? bond_term<true, REFC>(d, pr, ok) : bond_term<false>(d, pr, ok);
            }
        }
    }
    RowOut out{0.0f, 0.0f, 0u};
    if (TERMS) {
        // flags and band counts of the row's lanes
        unsigned fa = fl;
        float bsum = band;
        fa |= row_lane_u<LPR, 1>(fl);
        bsum += row_lane<LPR, 1>(band);
        if constexpr (LPR == 4) {
            fa |= row_lane_u<LPR, 2>(fl) | row_lane_u<LPR, 3>(fl);
            bsum += row_lane<LPR, 2>(band);
            bsum += row_lane<LPR, 3>(band);
        }
        // the bond terms in the others' index order: other j is pair
        // O + 1 + j, held by lane (O + 1 + j) % LPR in its slot / LPR
        float bv[A - 1];
#pragma unroll
        for (int j = 0; j < A - 1; ++j) {
            constexpr int dummy = 0;
            (void)dummy;
            const int pj = O + 1 + j;
            const int tj = pj / LPR;
            float v = 0.0f;
            switch (pj % LPR) {
            case 0: v = bt[tj]; break;
            case 1: v = row_lane<LPR, 1>(bt[tj]); break;
            case 2: if constexpr (LPR == 4) v = row_lane<LPR, 2>(bt[tj]); break;
            default: if constexpr (LPR == 4) v = row_lane<LPR, 3>(bt[tj]); break;
            }
            bv[j] = v;
        }
        const float bond = torch_row_sum_r<A - 1>(bv, [](float x) { return x; });
        out = row_reward<A, FAST, REFC>(ta, td, (fa & 5u) != 0u, (fa & 10u) != 0u, bsum, bond,
                                        pr, ok);
    }
    return out;
}

// ---------------------------------------------------------- helper wave
// Grids of at most one env-block per CU (16384 envs x 3 agents: 256 blocks of
// 3 waves, a quarter of the SIMDs idle) get a fourth wave per block on the
// idle SIMD. While waves 0..A-1 stage, move and observe, it draws the fresh
// obstacles of every env of the block (the native re-init's Philox draws) and
// computes the fresh env's agent-obstacle pairs (formation agents against
// those obstacles; agent a between the block barriers a and a+1, so it never
// holds a barrier back). After the observation barrier it re-initialises and
// re-observes the finished envs alone - the target and agent-agent pairs from
// the formation template (marlnav_formation_obs), the obstacle pairs from its
// own table - while wave 0 runs the per-env phase: the finished-env tail
// shrinks to copies and blends, and the draws leave the main waves' stage.

// fresh obstacles of env l (lane) of the block: its NB Philox blocks
template <int O>
__device__ __forceinline__ void helper_draws(const MarlnavParams &pr, uint64_t sidx, uint64_t gid,
                                             float (&fo)[2 * O])
{
#pragma unroll
    for (int jb = 0; jb < (O + 1) / 2; ++jb) {
        float v[4];
        native_obst_draws(pr.seed, sidx, gid, jb, pr.obs_range_x, pr.obs_mean_x, pr.obs_range_y,
                          pr.obs_mean_y, v);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (2 * jb + k / 2 < O) fo[4 * jb + k] = v[k];
    }
}

// the fresh env's pairs of formation agent a with its O fresh obstacles (the
// values native_pair_item computes for a clean env), into fr (E, A, 2O)
template <int A, int O>
__device__ __forceinline__ void helper_fresh_pairs(const float *__restrict__ gform, int a,
                                                   const float (&fo)[2 * O], float cap, float *fr,
                                                   int l)
{
    const float fx = gform[5 * a], fy = gform[5 * a + 1];
    const float fdx = gform[5 * a + 2], fdy = gform[5 * a + 3];
    bool cok = coord_ok(fx) && coord_ok(fy);
#pragma unroll
    for (int j = 0; j < 2 * O; ++j) cok = cok && coord_ok(fo[j]);
    float *o = fr + (l * A + a) * 2 * O;
    bool unused = true;
    if (__ballot(!cok) == 0ull) {
#pragma unroll
        for (int j = 0; j < O; ++j) {
            const float d = pair_dist<true>(fx, fy, fo[2 * j], fo[2 * j + 1], unused);
            o[j] = pair_angle<true>(fx, fy, fo[2 * j], fo[2 * j + 1], fdx, fdy, d, cap, unused);
            o[O + j] = d;
        }
    } else {
#pragma unroll
        for (int j = 0; j < O; ++j) {
            const float d = pair_dist<false>(fx, fy, fo[2 * j], fo[2 * j + 1], unused);
            o[j] = pair_angle<false>(fx, fy, fo[2 * j], fo[2 * j + 1], fdx, fdy, d, cap, unused);
            o[O + j] = d;
        }
    }
}

// The helper wave's finished-env tail (environment.py:76-90, 104-105): the
// finished set (the test wave 0's per-env phase makes), each finished env's
// cleanliness (every blended agent coordinate, the target and the obstacles
// equal to their fresh values, i.e. no non-finite old value: then the
// template and the helper's pairs describe the re-initialised env), then one
// item per (env, row, pair) - copied when clean, computed (native_pair_item)
// otherwise - and per state float / target / obstacle block (native_rest_item).
template <int A, int O, int E, int D>
__device__ __forceinline__ void helper_tail(KArgsK *kl, const BlockEnvs<A, O, D> &ev,
                                            const float *form, const float *pre, const float *fr,
                                            const float2 *__restrict__ tpl, const float4 *red,
                                            const float *sn, const uint8_t *tm, int ne,
                                            const MarlnavParams &pr, int lane)
{
    bool fin = false;
    if (lane < ne) {
        unsigned any_col = 0u;
#pragma unroll
        for (int i = 0; i < A; ++i) any_col |= __float_as_uint(red[A * lane + i].z) & 1u;
        fin = sn[lane] + 1.0f > pr.trunc_after || any_col != 0u || tm[lane] != 0;
    }
    const uint64_t fm = __ballot(fin);
    if (!fm) return;
    const int nfin = (int)__popcll(fm);
    bool cl = false;
    if (lane < nfin) {
        const int c = list_code(MaskList{fm}, lane, 0, nfin - 1);
        const float *s = ev.state(c);
        cl = true;
#pragma unroll
        for (int a = 0; a < A; ++a)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                cl = cl && __float_as_uint(blend_in(s[5 * a + k], form[5 * a + k])) ==
                               __float_as_uint(form[5 * a + k]);
        const float *t = ev.targ(c);
        cl = cl && __float_as_uint(blend_in(t[0], form[5 * A])) == __float_as_uint(form[5 * A]);
        cl = cl && __float_as_uint(blend_in(t[1], form[5 * A + 1])) ==
                       __float_as_uint(form[5 * A + 1]);
        const float *ob = ev.obst(c);
#pragma unroll
        for (int i = 0; i < 2 * O; ++i)
            cl = cl && __float_as_uint(blend_in(ob[i], pre[i * E + c])) ==
                           __float_as_uint(pre[i * E + c]);
    }
    const uint64_t cm = __ballot(cl);  // bit fe: finished env fe is clean
    using IT = NativeItems<A, O>;
    constexpr int NI = IT::NPAIR + IT::NREST;
    const float cap = pr.cap_distance;
    for (int base = 0; base < nfin * NI; base += 64) {
        const int i = base + lane;
        const bool on = i < nfin * NI;
        const int ic = on ? i : 0;
        const int fe = ic / NI, kk = ic - fe * NI;
        const int c = list_code(MaskList{fm}, fe, base / NI, min((base + 63) / NI, nfin - 1));
        if (kk < IT::NPAIR) {
            if ((cm >> fe) & 1ull) {
                if (on) {
                    const int ag = kk / IT::NP, p = kk - ag * IT::NP;
                    float *o = ev.row(c, ag);
                    if (p >= 1 && p <= O) {
                        const float *q = fr + (c * A + ag) * 2 * O;
                        o[1 + p] = q[p - 1];
                        o[1 + O + p] = q[O + p - 1];
                    } else {
                        const int m = p == 0 ? 0 : p - O;  // template column: 0 target, 1 + other
                        const float2 t = tpl[ag * A + m];
                        const int sa = p == 0 ? 0 : 2 + 2 * O + (m - 1);
                        const int sd = p == 0 ? 1 : 2 + 2 * O + (A - 1) + (m - 1);
                        o[sa] = t.y < cap ? 0.0f : t.x;  // the cap (environment.py:172-177)
                        o[sd] = t.y;
                    }
                }
            } else {
                native_pair_item<A, O, E>(kl, ev, form, pre, c, kk, on, cap);
            }
        } else if (on) {
            native_rest_item<A, O, E>(kl, ev, form, pre, c, kk - IT::NPAIR);
        }
    }
}

// Phases (one block barrier after each of the first four): stage | move +
// coordinate check | observe into LDS rows | per-env phase on wave 0 while
// waves 1..A-1 re-initialise and re-observe the finished envs (native
// re-init; none in most blocks) | rows and states stream out of LDS.
template <int A, int O, bool OBS_ONLY, bool NOISY, int LPR = 1, bool HELP = false>
__global__ void __launch_bounds__(64 * (A + HELP))
    block_kernel(float *h_states, const float *h_actions, const float *h_obstacles,
                 const float *h_target, const float *h_step_num, const uint8_t *h_terminates,
                 int64_t h_P, KArgs k)
{
    using BP = BlockPlan<A, O, LPR, HELP>;
    static_assert(!HELP || (!OBS_ONLY && !NOISY), "the helper serves the native re-init step");
    constexpr int E = BP::E, R = BP::R, D = BP::D, NT = BP::NT + (HELP ? 64 : 0);
    (void)k;  // read through kargs_late<kHotKargsOff>()
    extern __shared__ __attribute__((aligned(16))) float lds[];
#if MARLNAV_STAMPS
    unsigned long long t_entry;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_entry));
#endif
    const int tid = (int)threadIdx.x;
    const unsigned lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // agent of this wave
    const bool hw = HELP && w == A;  // the helper wave (no agent)
    const int64_t blk = blockIdx.x;
    const int64_t gw = blk * (A + HELP) + w;  // stamps slot
    KArgsK *K = kargs_late<kHotKargsOff>();
    const int64_t P = h_P;
    // launch_block's grid is exactly ntiles blocks: no exit test. The staging
    // pointers come preloaded in SGPRs; the rest are read from KArgs.
    StepPtrs b = load_ptrs(K);
    b.states = h_states;
    b.actions = h_actions;
    b.obstacles = const_cast<float *>(h_obstacles);
    b.target = const_cast<float *>(h_target);
    b.step_num = const_cast<float *>(h_step_num);
    b.terminates = const_cast<uint8_t *>(h_terminates);
    STAMP(0);
    float *st = lds + BP::ST;
    const int64_t e0 = blk * E;
    const int ne = (int)((P - e0) < E ? (P - e0) : E);
    const bool full = ne == E;

    // ---- this wave's actions (lane l: agent w of env l) into its own LDS
    // slots by LDS-DMA issued before the block's spans: the wave waits for
    // them alone (vmcnt = the span instructions it issued after them) and
    // evaluates the heading's sin/cos while the spans are still in flight,
    // not after the stage barrier
    float *actw = lds + BP::ACTW + 2 * E * w;  // x at [l], y at [E + l]
    if (!OBS_ONLY && full && (int)lane < E && !hw) {
        const float *pa = h_actions + ((e0 + lane) * A + w) * 2;
        __builtin_amdgcn_global_load_lds(pa, (LdsVoid *)actw, 4, 0, 0);
        __builtin_amdgcn_global_load_lds(pa + 1, (LdsVoid *)(actw + E), 4, 0, 0);
    }
    // ---- stage the block (spans spread over the waves: span k by wave k % A)
    using BS = BlockSpans<A, O, LPR>;
    static_assert(BS::NB[0] == R * 20 && BS::NB[1] == E * O * 8 && BS::NB[2] == E * 8 &&
                      BS::NB[3] == E * 4 && BS::NB[4] == E && BS::NB[5] == (5 * A + 2) * 4,
                  "span table and LDS plan agree");
    if (full) {
        block_glds<BS::NB[0]>(BS::K[0], A, w, b.states + e0 * (A * 5), st, lane);
        block_glds<BS::NB[1]>(BS::K[1], A, w, b.obstacles + e0 * (O * 2), lds + BP::OB, lane);
        block_glds<BS::NB[2]>(BS::K[2], A, w, b.target + e0 * 2, lds + BP::TG, lane);
        if (!OBS_ONLY) {
            block_glds<BS::NB[3]>(BS::K[3], A, w, b.step_num + e0, lds + BP::SN, lane);
            block_glds<BS::NB[4]>(BS::K[4], A, w, b.terminates + e0, lds + BP::TM, lane);
            if (b.formation)
                block_glds<BS::NB[5]>(BS::K[5], A, w, b.formation, lds + BP::FORM, lane);
        }
    } else {
        const int nr = ne * A;
        block_copy(b.states + e0 * (A * 5), st, nr * 5, tid, NT);
        if (!OBS_ONLY && (int)lane < ne && !hw) {  // (each lane its own slots: no barrier)
            const float *pa = h_actions + ((e0 + lane) * A + w) * 2;
            actw[lane] = pa[0];
            actw[E + lane] = pa[1];
        }
        block_copy(b.obstacles + e0 * (O * 2), lds + BP::OB, ne * O * 2, tid, NT);
        block_copy(b.target + e0 * 2, lds + BP::TG, ne * 2, tid, NT);
        if (!OBS_ONLY) {
            block_copy(b.step_num + e0, lds + BP::SN, ne, tid, NT);
            block_copy(b.terminates + e0, reinterpret_cast<uint8_t *>(lds + BP::TM), ne, tid, NT);
            if (b.formation) block_copy(b.formation, lds + BP::FORM, 5 * A + 2, tid, NT);
        }
    }
    const MarlnavParams pr = load_params(K);
    const bool wt = (pr.flags & kWriteThroughFlag) != 0;  // written-through outputs
    // native (non-noisy) re-init: waves 1..A-1 take the finished envs while
    // wave 0 runs the per-env phase (below)
    const bool overlap = !OBS_ONLY && !NOISY && !K->a.b.fresh_states;
    // (one Philox block per thread at most: at A3/O8 the two passes cost the
    // stage phase more than they save, 131072x3x8 18.4 -> 19.0 us)
    constexpr bool kPre = E * ((O + 1) / 2) <= NT;
    // (HELP: the helper wave's fresh obstacles of env `lane`, kept in
    // registers from the draws until its agent-obstacle pairs are done)
    float hfo[HELP ? 2 * O : 1];
    (void)hfo;
    if constexpr (HELP) {
        if (hw && overlap) {
            KArgsK *kl = kargs_late<kHotKargsOff>();
            float(&fo)[2 * O] = reinterpret_cast<float(&)[2 * O]>(hfo);
            helper_draws<O>(pr, kl->a.step_idx, (uint64_t)(kl->a.env_offset + e0 + lane), fo);
            float *pre = lds + BP::FRESH;
#pragma unroll
            for (int i = 0; i < 2 * O; ++i)
                if ((int)lane < ne) pre[i * E + lane] = fo[i];
            helper_fresh_pairs<A, O>(b.formation, 0, fo, pr.cap_distance, lds + BP::FR, (int)lane);
        }
    } else if (kPre && overlap && !(MARLNAV_AB & 256)) {  // (AB 256: timing only, no draws)
        // the fresh obstacles of every env of the block (its Philox draws
        // depend only on seed, step and env id), drawn while the staging
        // loads are in flight: a finished env's re-init then reads them
        // instead of drawing after the per-env barrier, where the draws sat
        // on the block's critical path (65536x3x3: 0.25 us of 0.63)
        KArgsK *kl = kargs_late<kHotKargsOff>();
        const uint64_t sidx = kl->a.step_idx, g0 = (uint64_t)(kl->a.env_offset + e0);
        constexpr int NB = (O + 1) / 2;
        float *pre = lds + BP::FRESH;
#pragma unroll
        for (int k2 = 0; k2 * NT < E * NB; ++k2) {
            const int i = tid + k2 * NT;
            const int l = i % E, jb = i / E;
            if (((k2 + 1) * NT <= E * NB || i < E * NB) && l < ne) {
                float v[4];
                native_obst_draws(pr.seed, sidx, g0 + l, jb, pr.obs_range_x, pr.obs_mean_x,
                                  pr.obs_range_y, pr.obs_mean_y, v);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (2 * jb + k / 2 < O) pre[(4 * jb + k) * E + l] = v[k];
            }
        }
    }
    // the heading's sin/cos (environment.py:113-115, 131-137), under the
    // remaining staging latency
    float sn = 0.0f, c = 1.0f, a1 = 0.0f;
    if (!OBS_ONLY && !hw) {
        if (full) {
            // span instructions this wave issued after its two action loads
            // (BlockSpans: the same table as the issue sites above)
            int n = 0;
#pragma unroll
            for (int ww = 0; ww < A; ++ww)
                if (w == ww) n = b.formation ? BS::after_actions(ww, true) : BS::after_actions(ww, false);
            wait_vmcnt(n);
        }
        float a0 = actw[lane / LPR];  // (the LPR lanes of a row: the same agent)
        a1 = actw[E + lane / LPR];
        if (pr.flags & MARLNAV_SCALE_ACTIONS) {  // ActionScaler (utils.py:546-547)
            KArgsK *kl = kargs_late<kHotKargsOff>();
            a0 = kl->p.act_scale[0] * a0 + kl->p.act_mean[0];
            a1 = kl->p.act_scale[1] * a1 + kl->p.act_mean[1];
        }
        sincos_k(clamp_t(a0, -kPiF, kPiF), &sn, &c);
    }
    const int l = (int)lane / LPR;   // env of this lane's row within the block
    const int sub = (int)lane % LPR;  // the lane's place in its row's lane group
    const int r = l * A + (hw ? 0 : w);  // row of this lane (the helper has none)
    const bool row_on = l < ne && !hw;
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
    if (full) {
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
        const float ndx = c * dx + (-sn) * dy;
        const float ndy = sn * dx + c * dy;
        float *s = st + 5 * r;
        const float v = clamp_t(s[4] + clamp_t(a1, pr.min_accel, pr.max_accel), pr.min_speed,
                                pr.max_speed);
        ox = ox + ndx * v;
        oy = oy + ndy * v;
        dx = ndx;
        dy = ndy;
        if (row_on && sub == 0) {
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
    if constexpr (HELP) {  // agent 1's fresh pairs, between the stage and move barriers
        if (hw && overlap && A > 1)
            helper_fresh_pairs<A, O>(b.formation, 1, reinterpret_cast<float(&)[2 * O]>(hfo),
                                     pr.cap_distance, lds + BP::FR, (int)lane);
    }
    if (full) {
        if (!hw) {  // (the helper's share of the obstacle / target check still counts)
            crange.add(ox);
            crange.add(oy);
        }
        // one word for the block, written only by waves that found one (all
        // write 1: a benign race); read once after the barrier
        const bool bad = __ballot(!crange.ok()) != 0ull;
        if (lane == 0 && bad) *bad_word = 1;
    }
    __syncthreads();
    STAMP(2);
    // the moved states are final except in finished envs (re-stored below)
    const bool fast = full && *bad_word == 0;

    // ---- observations of the moved state + reward terms (:99-100)
    float4 *red = reinterpret_cast<float4 *>(lds + BP::RED);
    float *obs_rows = lds + BP::OBS;
    // agent-pair symmetry (block_observe_sym): FAST A3 blocks of A/B builds
    // with MARLNAV_SYM (no faster than the per-direction rows: DESIGN.md §5)
    constexpr bool kSym = A == 3 && LPR == 1 && !HELP && MARLNAV_SYM;
    const bool refc = !MARLNAV_AB_NOREFC && pr.bond_sharpness == 1.0f && pr.max_at_prop_d == 2.0f;
    bool sym = false;
    // finished envs re-initialised and re-observed inside the symmetric
    // observation phase (block_observe_sym EARLY): native non-noisy re-init
    // with the stage-time draws
    bool early = false;
    if constexpr (kSym) {
        if (__builtin_expect(fast, 1)) {
            float2 *pt = reinterpret_cast<float2 *>(lds + BP::PT);
            const float *obe = lds + BP::OB + 2 * O * l, *tge = lds + BP::TG + 2 * l;
            if constexpr (!OBS_ONLY && kPre && !(MARLNAV_AB & 1) && MARLNAV_EARLY) {
                early = overlap;
                if (early) {
                    const EarlyReinit er{kargs_late<kHotKargsOff>(), lds + BP::FORM, lds + BP::FRESH,
                                         lds + BP::SN, reinterpret_cast<const uint8_t *>(lds + BP::TM),
                                         lds + BP::OB, lds + BP::TG, e0, ne};
                    if (refc)
                        block_observe_sym<A, O, true, true, true>(st, obe, tge, l, w, ox, oy, dx, dy,
                                                                  obs_rows, pt, red, pr, er);
                    else
                        block_observe_sym<A, O, true, false, true>(st, obe, tge, l, w, ox, oy, dx,
                                                                   dy, obs_rows, pt, red, pr, er);
                }
            }
            if (!early) {
                if (refc)
                    block_observe_sym<A, O, !OBS_ONLY, true>(st, obe, tge, l, w, ox, oy, dx, dy,
                                                             obs_rows, pt, red, pr);
                else
                    block_observe_sym<A, O, !OBS_ONLY, false>(st, obe, tge, l, w, ox, oy, dx, dy,
                                                              obs_rows, pt, red, pr);
            }
            sym = true;
        }
    }
    if constexpr (LPR > 1) {
        if (row_on) {
            const float *se = st + 5 * A * l, *obe = lds + BP::OB + 2 * O * l, *tge = lds + BP::TG + 2 * l;
            float *rw = obs_rows + r * D;
            RowOut ro;
            if (__builtin_expect(fast, 1) && refc)
                ro = observe_row_lpr<A, O, LPR, !OBS_ONLY, true, true>(se, obe, tge, w, sub, ox, oy,
                                                                       dx, dy, rw, pr);
            else if (__builtin_expect(fast, 1))
                ro = observe_row_lpr<A, O, LPR, !OBS_ONLY, true, false>(se, obe, tge, w, sub, ox, oy,
                                                                        dx, dy, rw, pr);
            else
                ro = observe_row_lpr<A, O, LPR, !OBS_ONLY, false, false>(se, obe, tge, w, sub, ox,
                                                                         oy, dx, dy, rw, pr);
            if (!OBS_ONLY && sub == 0)
                red[r] = make_float4(ro.r_miss, ro.r_hit, __uint_as_float(ro.flags), 0.0f);
        }
        sym = true;  // (done)
    }
    if (!sym && row_on) {
        float rowv[D];
        RowOut ro;
        bool unused = true;
        if (__builtin_expect(fast, 1) && refc)
            ro = observe_row_own<A, O, !OBS_ONLY, true, true>(st + 5 * A * l, lds + BP::OB + 2 * O * l,
                                                              lds + BP::TG + 2 * l, w, ox, oy, dx,
                                                              dy, rowv, pr, unused);
        else if (__builtin_expect(fast, 1))
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
    if constexpr (HELP) {  // agents 2.. fresh pairs, under the observation phase
        if (hw && overlap)
#pragma unroll
            for (int a = 2; a < A; ++a)
                helper_fresh_pairs<A, O>(b.formation, a, reinterpret_cast<float(&)[2 * O]>(hfo),
                                         pr.cap_distance, lds + BP::FR, (int)lane);
    }
    __syncthreads();
    STAMP(3);
    float *gobs = in_sgpr(b.obs + e0 * (A * D));
    if (OBS_ONLY) block_store(gobs, obs_rows, nrow * D, tid, NT, wt);
    const bool norm = !OBS_ONLY && (pr.flags & MARLNAV_WRITE_OBS_NORM);
    if (!OBS_ONLY) {
        int *list = reinterpret_cast<int *>(lds + BP::LIST);
        int *flg = reinterpret_cast<int *>(lds + BP::FLG);
        const BlockEnvs<A, O, D> ev{st, lds + BP::OB, lds + BP::TG, obs_rows, e0};
        // ---- per-env reductions, terminal logic (wave 0, one lane per env)
        // (env le = lane here: one lane per env, whatever LPR)
        const int le = (int)lane;
        if (w == 0) {
            const bool env_on = le < ne;
            bool fin = false, tr_l = false, co_l = false, ta_l = false;
            if (env_on) {
                const int64_t e = e0 + le;
                float4 rr[A];
#pragma unroll
                for (int i = 0; i < A; ++i) rr[i] = red[A * le + i];
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
                STAMPX(0);  // (wave 0: the reward terms read)
                const float rsum = torch_row_sum_r<A>(rv, [](float x) { return x; });
                if (!(MARLNAV_AB & 1024))  // (AB 1024: timing only, no per-env stores)
                out_el(b.reward, e, rsum / (float)A);              // torch.mean (:233)

                float step_num = lds[BP::SN + le] + 1.0f;           // :96
                const bool truncated = step_num > pr.trunc_after;  // :97
                const bool term_old = reinterpret_cast<const uint8_t *>(lds + BP::TM)[le] != 0;
                const bool terminated = any_col || term_old;       // :213-214
                if (!(MARLNAV_AB & 1024)) {
                out_el(b.terminates, e, (uint8_t)(!term_old && all_in));  // :218-219
                out_el(b.terminated, e, (uint8_t)terminated);
                out_el(b.truncated, e, (uint8_t)truncated);
                }
                fin = truncated || terminated;                     // :102-104
                if (NOISY && fin) {  // noisy native re-init: serial per env
                    KArgsK *kl = kargs_late<kHotKargsOff>();
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
                        float *obl = lds + BP::OB + 2 * O * le;
                        float *tgl = lds + BP::TG + 2 * le;
                        native_fresh_env<NOISY>(A, O, p, lds + BP::FORM,
                                                (uint64_t)(kl->a.env_offset + e), kl->a.step_idx,
                                                st + 5 * A * le, obl, tgl);
                        float *gob = kl->a.b.obstacles;
                        for (int i = 0; i < 2 * O; ++i) out_el(gob, e * O * 2 + i, obl[i]);
                        out_el(kl->a.b.target, 2 * e, tgl[0]);
                        out_el(kl->a.b.target, 2 * e + 1, tgl[1]);
                    }
                }
                if (!(MARLNAV_AB & 1024))
                out_el(b.step_num, e, fin ? blend_in(step_num, 0.0f) : step_num);
                tr_l = truncated;
                co_l = any_col;
                ta_l = all_in;
            }
            STAMPX(1);  // (wave 0: the per-env outputs issued)
            const uint64_t finmask = __ballot(fin);
            if (fin)
                list[__builtin_amdgcn_mbcnt_hi((unsigned)(finmask >> 32),
                                               __builtin_amdgcn_mbcnt_lo((unsigned)finmask, 0u))] = le;
            const unsigned c_trunc = __popcll(__ballot(tr_l));
            const unsigned c_col = __popcll(__ballot(co_l));
            const unsigned c_tar = __popcll(__ballot(ta_l));
            if (lane == 0) {
                flg[0] = (int)__popcll(finmask);
                if ((c_trunc | c_col | c_tar) && !(MARLNAV_AB & 512)) {  // (AB 512: timing only)
                    KArgsK *kl = kargs_late<kHotKargsOff>();
                    uint64_t *cnt = kl->a.b.counters;
                    const int64_t slots = kl->a.waves;
                    if (cnt) {
                        const int64_t sl = blk < slots ? blk : blk % slots;
                        if (c_trunc) atomicAdd((unsigned long long *)&cnt[0 * slots + sl], (unsigned long long)c_trunc);
                        if (c_col) atomicAdd((unsigned long long *)&cnt[1 * slots + sl], (unsigned long long)c_col);
                        if (c_tar) atomicAdd((unsigned long long *)&cnt[2 * slots + sl], (unsigned long long)c_tar);
                    }
                }
            }
            STAMPX(2);  // (wave 0: list, counts and counters done)
        } else if (HELP && overlap) {
            // ---- the helper wave's finished-env tail (waves 1..A-1 idle)
            if constexpr (HELP) {
                if (hw && !(MARLNAV_AB & 1))
                    helper_tail<A, O, E, D>(kargs_late<kHotKargsOff>(), ev, lds + BP::FORM,
                                            lds + BP::FRESH, lds + BP::FR,
                                            reinterpret_cast<const float2 *>(K->a.b.formation_obs),
                                            red, lds + BP::SN,
                                            reinterpret_cast<const uint8_t *>(lds + BP::TM), ne, pr,
                                            (int)lane);
            }
        } else if (overlap && !early) {
            // ---- waves 1..A-1, while wave 0 runs the per-env phase: the
            // finished set from the inputs wave 0 uses (red flags, step_num,
            // terminates), then the native re-init (:104) and re-observation
            // (:105) of those envs. Disjoint LDS: wave 0 reads red/SN/TM; this
            // writes the states, obstacles, target and rows of finished envs.
            bool fin = false;
            if (le < ne) {
                unsigned any_col = 0u;
#pragma unroll
                for (int i = 0; i < A; ++i) any_col |= __float_as_uint(red[A * le + i].z) & 1u;
                fin = lds[BP::SN + le] + 1.0f > pr.trunc_after || any_col != 0u ||
                      reinterpret_cast<const uint8_t *>(lds + BP::TM)[le] != 0;
            }
            const uint64_t fm = __ballot(fin);
            STAMPX(0);
            if (fm && !(MARLNAV_AB & 1)) {
                STAMPX(1);
                reinit_reobs_native<A, O, kPre ? E : 0>(kargs_late<kHotKargsOff>(), ev,
                                                        lds + BP::FORM, MaskList{fm},
                                                        (int)__popcll(fm), pr.cap_distance,
                                                        tid - 64, NT - 64, lds + BP::FRESH);
                STAMPX(2);
            }
        }
        __syncthreads();
        STAMP(4);
        const int nfin = flg[0];
        if (nfin && !overlap) {
            // ---- reference-RNG / noisy re-init (:104; noisy: done above by
            // wave 0) and observations of the re-initialised envs (:105)
            if (!NOISY) {
                reinit_block<A, O>(kargs_late<kHotKargsOff>(), ev, lds + BP::FORM, list, nfin, tid, NT);
                __syncthreads();
            }
            reobs_block<A, O>(ev, list, nfin, pr.cap_distance, tid, NT);
            __syncthreads();
        }
    }
    STAMP(5);
    if (!OBS_ONLY && full && !norm) {  // ---- stream the block out
        if (!(MARLNAV_AB & 2))
        block_store2<E * A * D, E * A * 5, NT>(gobs, obs_rows, in_sgpr(b.states_out + e0 * (A * 5)),
                                               st, tid, wt);  // (E = 64: whole 16-byte pieces)
    } else if (!OBS_ONLY && full && NT % D == 0) {
        // ---- the same with the fused ObsNormalizer (utils.py:519-532):
        // thread tid only ever meets feature tid % D (NT is a multiple of D),
        // so its mean and scale are loaded once; every LDS read and every
        // division is issued ahead of the stores
        block_store2<E * A * D, E * A * 5, NT>(gobs, obs_rows, in_sgpr(b.states_out + e0 * (A * 5)),
                                               st, tid, wt);
        KArgsK *kl = kargs_late<kHotKargsOff>();
        const int kk = tid % D;
        const float m = kl->a.b.norm_mean[kk], sc = kl->a.b.norm_scale[kk];
        float *gn = kl->a.b.obs_norm + e0 * (A * D);
        constexpr int K = E * A * D / NT;
        static_assert(E * A * D % NT == 0, "whole passes");
        float v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = obs_rows[tid + k * NT];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = (v[k] - m) / sc;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (kWtOut && wt)
                wt_st(out_buf(gn, E * A * D * 4), 4u * (tid + k * NT), v[k]);
            else
                out_st<kNtRows>(gn + tid + k * NT, v[k]);
        }
    } else if (!OBS_ONLY) {
        block_store(gobs, obs_rows, nrow * D, tid, NT, wt);
        if (norm) {
            // mean and scale staged in LDS once (the reward-term slots are
            // free after the per-env phase), then one pass over the rows
            KArgsK *kl = kargs_late<kHotKargsOff>();
            float *ms = lds + BP::RED;
            static_assert(4 * R >= 2 * D, "mean and scale fit the reward-term slots");
            if (tid < D) {
                ms[tid] = kl->a.b.norm_mean[tid];
                ms[D + tid] = kl->a.b.norm_scale[tid];
            }
            __syncthreads();
            float *gn = kl->a.b.obs_norm + e0 * (A * D);
            const OutBuf nb = out_buf(gn, 4u * nrow * D);
#pragma unroll 4
            for (int i = tid; i < nrow * D; i += NT) {
                const int kk = i % D;
                const float v = (obs_rows[i] - ms[kk]) / ms[D + kk];
                if (kWtOut && wt)
                    wt_st(nb, 4u * i, v);
                else
                    gn[i] = v;
            }
        }
        block_store(in_sgpr(b.states_out + e0 * (A * 5)), st, nrow * 5, tid, NT, wt);
    }
    STAMP(6);
#if MARLNAV_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(7);
    if (lane == 0) {
        *STAMP_PTR((size_t)gw * 24 + 16) = t_entry;
        *STAMP_PTR((size_t)gw * 24 + 17) = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        *STAMP_PTR((size_t)gw * 24 + 18) = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
        *STAMP_PTR((size_t)gw * 24 + 19) = OBS_ONLY ? 0u : (unsigned)reinterpret_cast<const int *>(lds + BP::FLG)[0];
    }
#endif
    (void)gw;
}
