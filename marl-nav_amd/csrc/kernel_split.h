// kernel_split.h - pair-split kernel (LPR lanes per agent row: A16/O32, small A3 grids).
// Part of libmarlnav.so: included once, by marlnav_step.hip (one translation
// unit), inside its anonymous namespace.
#pragma once

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

// The workgroup's finished envs as one list built by wave 0's per-env
// phase (workgroup-spread shapes): env codes wave * EPW + env.
struct FlatFinList {
    const int *slot;
    int n;
    __device__ int total() const { return n; }
    __device__ int operator[](int fe) const { return slot[fe]; }
};

// Finished envs re-initialised and re-observed by the whole workgroup
// (after one block barrier) instead of by their own wave: pays where an
// env's re-observation is long (measured: A3/O8 and A16/O32 faster, A3/O3
// slower).
template <int A, int O>
constexpr bool kSplitSpread = A * (1 + O + (A - 1)) >= 32;

// Spread re-init of many-obstacle shapes (O > 8: reinit_block, then the
// re-observation) with the formation and its observation template staged in
// LDS (kernel_reinit.h: reobs_block_tpl).
template <int A, int O>
constexpr bool kSplitTpl = kSplitSpread<A, O> && O > 8;

// Where the per-row reward terms are finished: on each row's leader lane at
// the end of the pair phase (few-obstacle shapes: 1024x3x8 5.09 -> 5.00 us,
// A/B in profiles/r03_ab_logs2.txt), or, for the workgroup-spread
// many-obstacle shapes, on wave 0 after the per-env barrier, one lane per row
// (4096x16x32 11.76 vs 11.84 us on the row leaders). MARLNAV_SPLIT_RR_LEADER
// (A/B builds) forces the row leaders everywhere.
template <int A, int O>
constexpr bool kSplitRRLeader = !kSplitSpread<A, O> || O <= 8 || MARLNAV_SPLIT_RR_LEADER;

// ... re-initialised and re-observed in one pass (reinit_reobs_tpl: the
// workgroup's threads cover whole obstacle columns)
template <int A, int O>
constexpr bool kSplitTplPass = kSplitTpl<A, O> && (64 * kWavesPerBlock) % O == 0;

// Extra LDS cycles of the workgroup-spread row-reward read (kernel_split.h,
// wave 0, lane = tile cw * R + row rw, reading the row's K bond terms at
// tile base cw * F + BOND, row stride K, one ds_read_b32 per term): banks are
// (dword address) mod 32, lanes conflict within each 32-lane half
// (MI355X_MICROARCH.md §LDS). Round 2 left F = 40 mod 64 at A16/O32, a 2-way
// conflict on every such read (+30 cycles per workgroup and step, the whole
// rise of SQ_LDS_BANK_CONFLICT that round: 131k -> 166k per launch).
__host__ __device__ constexpr int split_bond_conflicts(int BOND, int F, int K, int R)
{
    int extra = 0;
    const int tiles = 64 / R < kWavesPerBlock ? 64 / R : kWavesPerBlock;
    for (int j = 0; j < K; ++j)
        for (int half = 0; half < 2; ++half) {
            int worst = 1;
            for (int bank = 0; bank < 32; ++bank) {
                int n = 0;
                for (int l = 32 * half; l < 32 * half + 32; ++l) {
                    const int cw = l / R, rw = l % R;
                    if (cw >= tiles) continue;
                    const int a = cw * F + BOND + K * rw + j;
                    n += (a % 32 == bank) ? 1 : 0;
                }
                worst = n > worst ? n : worst;
            }
            extra += worst - 1;
        }
    return extra;
}

// the smallest tile padding (floats, multiple of 4) with the fewest such
// conflicts
__host__ __device__ constexpr int split_tile_pad(int BOND, int F0, int K, int R)
{
    if (K <= 0) return 0;
    int best = 0, best_c = split_bond_conflicts(BOND, F0, K, R);
    for (int pad = 4; pad < 64 && best_c > 0; pad += 4) {
        const int c = split_bond_conflicts(BOND, F0 + pad, K, R);
        if (c < best_c) {
            best_c = c;
            best = pad;
        }
    }
    return best;
}

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
    // wave-tile stride, padded so that wave 0's one-lane-per-row read of
    // every tile's bond terms (row_reward, after the workgroup barrier) is
    // free of LDS bank conflicts (split_tile_pad)
    static constexpr int FLOATS = RED + 4 * R + split_tile_pad(BOND, RED + 4 * R, A - 1, R);
    // formation (5A + 2 floats) and its observation template (2A^2 floats),
    // staged for the spread re-init of kSplitTpl shapes
    static constexpr int NF = 5 * A + 2, NCP = NF + 2 * A * A;
    // after the waves' regions: finished-env counts and slots of the
    // workgroup, the `unclean` word (reinit_block), then (kSplitTpl) the
    // formation and template at FTP
    // (+ kWavesPerBlock * EPW step numbers and as many `terminates` flags:
    // the workgroup's per-env inputs, parked for wave 0's per-env phase)
    static constexpr int ENVIN = (kWavesPerBlock * (1 + EPW) + 1 + 3) & ~3;
    static constexpr int FTP = (ENVIN + 2 * kWavesPerBlock * EPW + 3) & ~3;
    // then (kSplitSpread shapes with O <= 8, native re-init) the fresh
    // obstacle draws of the workgroup's EW envs, component k of obstacle j of
    // env code c at PRE + (2j + k) * EW + c (native_obst_draw, device_math.h)
    static constexpr int EW = kWavesPerBlock * EPW;
    // (kSplitSpread shapes with O <= 8: the formation alone at FTP, for the
    // fused native re-init pass: MARLNAV_SPLIT_FORM_LDS)
    static constexpr int PRE = (FTP + (kSplitTpl<A, O> ? NCP : (kSplitSpread<A, O> && O <= 8 && MARLNAV_SPLIT_FORM_LDS ? NF : 0)) + 3) & ~3;
    static constexpr int BLK = PRE + (kSplitSpread<A, O> && O <= 8 ? 2 * O * EW : 0);
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

// The target pair takes a spare slot of lane LPR-1 when the other agents (or
// else the obstacles) do not divide over the LPR lanes: one pair body fewer per
// wave (A16/O32: 13 -> 12, A3/O8: 4 -> 3); the row leader reads the target
// angle/distance back from the LDS row.
template <int A, int O, int LPR>
constexpr bool kSplitTgtInAg = (A - 1) % LPR != 0;
template <int A, int O, int LPR>
constexpr bool kSplitTgtInOb = !kSplitTgtInAg<A, O, LPR> && O % LPR != 0;

// unroll factor of split_pairs' obstacle / other-agent loops (timing builds)

template <int A, int O, int LPR, bool TERMS, bool FAST, bool TFAST = false, bool SHARP1 = false>
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
    // obstacle and other-agent flags from the nearest one (d < r for some d
    // <=> min d < r; v_min ignores a NaN distance, which compares false
    // either way)
    float ob_min = __builtin_inff(), ag_min = __builtin_inff();
    // TFAST (FAST tiles, parameters inside the short sequences' guards,
    // kTermsFastFlag): the bond terms' divisions by the exact short sequences
    static_assert(!TFAST || FAST, "short divisions need the fast coordinate range");
    DivC d_sharp{1.0f, 1.0f};
    // SHARP1: bond_sharpness == 1 (the reference's constant, environment.py:
    // 66), where (d - ideal) / 1 is d - ideal exactly
    if constexpr (TERMS && TFAST && !SHARP1) d_sharp = make_divc(pr.bond_sharpness, ok);
    if constexpr (FAST && MARLNAV_PACKED_SPLIT && !(MARLNAV_AB & 64)) {
        // every slot's pair first - two per pair2_fast (pairs_fast); a slot
        // with no pair (j >= O, or kx >= A - 1 off the target lane) computes
        // a discarded one - then the row writes and terms of the loops below
        constexpr bool TS = !kSplitTgtInAg<A, O, LPR> && !kSplitTgtInOb<A, O, LPR>;
        constexpr int T0 = TS ? 1 : 0, N = T0 + SP::NOB + SP::NAG;
        float px[N], py[N], pd[N], pg[N];
        if constexpr (TS) {
            px[0] = tge[0];
            py[0] = tge[1];
        }
#pragma unroll
        for (int i = 0; i < SP::NOB; ++i) {
            const int j = q + LPR * i;
            const bool valid = O % LPR == 0 || j < O;
            const bool tgt = kSplitTgtInOb<A, O, LPR> && i == SP::NOB - 1 && q == TQ;
            const float *pt = tgt ? tge : obe + 2 * (valid ? j : 0);
            px[T0 + i] = pt[0];
            py[T0 + i] = pt[1];
        }
#pragma unroll
        for (int i = 0; i < SP::NAG; ++i) {
            const int kx = q + LPR * i;
            const bool valid = (A - 1) % LPR == 0 || kx < A - 1;
            const bool tgt = kSplitTgtInAg<A, O, LPR> && i == SP::NAG - 1 && q == TQ;
            const int m = valid ? kx + (kx >= a ? 1 : 0) : 0;
            const float *pt = tgt ? tge : sts + 5 * m;
            px[T0 + SP::NOB + i] = pt[0];
            py[T0 + SP::NOB + i] = pt[1];
        }
        pairs_fast<N>(ox, oy, dx, dy, px, py, cap, pd, pg);
        if constexpr (TS) {
            t.ta = pg[0];
            t.td = pd[0];
            if (q == 0) {
                orow[0] = pg[0];
                orow[1] = pd[0];
            }
        }
#pragma unroll
        for (int i = 0; i < SP::NOB; ++i) {
            const int j = q + LPR * i;
            const bool valid = O % LPR == 0 || j < O;
            const bool tgt = kSplitTgtInOb<A, O, LPR> && i == SP::NOB - 1 && q == TQ;
            const float d = pd[T0 + i], ang = pg[T0 + i];
            if (valid) {
                orow[2 + j] = ang;
                orow[2 + O + j] = d;
                if (TERMS) ob_min = __builtin_fminf(ob_min, d);
            } else if (tgt) {
                orow[0] = ang;
                orow[1] = d;
            }
        }
#pragma unroll
        for (int i = 0; i < SP::NAG; ++i) {
            const int kx = q + LPR * i;
            const bool valid = (A - 1) % LPR == 0 || kx < A - 1;
            const bool tgt = kSplitTgtInAg<A, O, LPR> && i == SP::NAG - 1 && q == TQ;
            const float d = pd[T0 + SP::NOB + i], ang = pg[T0 + SP::NOB + i];
            if (valid) {
                orow[2 + 2 * O + kx] = ang;
                orow[2 + 2 * O + (A - 1) + kx] = d;
                if (TERMS) {
                    ag_min = __builtin_fminf(ag_min, d);
                    t.band += (pr.agents_min_d < d && d < pr.agents_max_d) ? 1 : 0;
                    if constexpr (TFAST) {
                        const float sd = SHARP1 ? d - pr.ideal_dist
                                                : div_c(d - pr.ideal_dist, d_sharp, ok);
                        bond_row[kx] = recip_fast(1.0f + sd * sd, ok);
                    } else {
                        const float sd = (d - pr.ideal_dist) / pr.bond_sharpness;
                        bond_row[kx] = 1.0f / (1.0f + sd * sd);
                    }
                }
            } else if (tgt) {
                orow[0] = ang;
                orow[1] = d;
            }
        }
        if (TERMS)
            t.fl |= (ob_min < pr.ob_risk_dist ? 1u : 0u) | (ob_min < pr.ob_coll_dist ? 2u : 0u) |
                    (ag_min < pr.ag_risk_dist ? 4u : 0u) | (ag_min < pr.ag_coll_dist ? 8u : 0u);
        return t;
    }
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
#pragma unroll 64
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
                if (TERMS) ob_min = __builtin_fminf(ob_min, d);
            } else {
                orow[0] = ang;
                orow[1] = d;
            }
        }
    }
#pragma unroll 64
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
                    ag_min = __builtin_fminf(ag_min, d);  // flags after the loop, as for obstacles
                    t.band += (pr.agents_min_d < d && d < pr.agents_max_d) ? 1 : 0;
                    if constexpr (TFAST) {
                        const float sd = SHARP1 ? d - pr.ideal_dist
                                                : div_c(d - pr.ideal_dist, d_sharp, ok);
                        bond_row[kx] = recip_fast(1.0f + sd * sd, ok);
                    } else {
                        const float sd = (d - pr.ideal_dist) / pr.bond_sharpness;
                        bond_row[kx] = 1.0f / (1.0f + sd * sd);
                    }
                }
            }
        }
    }
    if (TERMS)
        t.fl |= (ob_min < pr.ob_risk_dist ? 1u : 0u) | (ob_min < pr.ob_coll_dist ? 2u : 0u) |
                (ag_min < pr.ag_risk_dist ? 4u : 0u) | (ag_min < pr.ag_coll_dist ? 8u : 0u);
    return t;
}

// one env code as a finished-env list (kernel_reinit.h passes)
struct OneEnv {
    int c;
    __device__ int operator[](int) const { return c; }
};

// ---- one env per wave (A16/O32 at LPR 4): the observation in two passes,
// so a finished env's wave can skip the bearings of the observation the
// re-initialisation discards (environment.py:99-105: rows of finished envs
// are replaced by the fresh env's) and spend them on the fresh env's rows
// instead, before the per-env barrier (kSplitOwn). Pass 1 computes every
// pair's distance (kept in registers), the reward flags, band and bond terms
// exactly as split_pairs does; pass 2 the bearings from those distances (the
// same pair_angle operations on the same inputs: bit for bit what
// split_pairs writes).
// The shapes that can run it (kSplitOwn: the instantiation that does,
// split_kernel's OWN; marlnav_step picks it for grids of at most
// kSplitOwnMaxEnvs envs, where it measured faster - at four waves per SIMD
// the SIMDs are VALU-saturated and moving a finished env's work from the
// workgroup's tail into its wave's observation saves no issue time).
template <int A, int O, int LPR>
constexpr bool kSplitOwnShape = kSplitTplPass<A, O> && 64 / LPR / A == 1;
template <int A, int O, int LPR, bool OWN>
constexpr bool kSplitOwn = kSplitOwnShape<A, O, LPR> && (OWN || MARLNAV_SPLIT_OWN);

template <int A, int O, int LPR>
struct SplitSlots {
    using SP = SplitPlan<A, O, LPR>;
    static constexpr int N = SP::NOB + SP::NAG;
};

template <int A, int O, int LPR, bool FAST, bool TFAST, bool SHARP1>
__device__ __forceinline__ SplitTerms split_dists(const float *__restrict__ sts,
                                                  const float *__restrict__ obe,
                                                  const float *__restrict__ tge, int a, int q,
                                                  float ox, float oy, float *__restrict__ bond_row,
                                                  const MarlnavParams &pr, bool &ok,
                                                  float (&dst)[SplitSlots<A, O, LPR>::N])
{
    using SP = SplitPlan<A, O, LPR>;
    constexpr int TQ = LPR - 1;
    SplitTerms t{0u, 0, 0.0f, 0.0f};
    float ob_min = __builtin_inff(), ag_min = __builtin_inff();
    static_assert(!TFAST || FAST, "short divisions need the fast coordinate range");
    DivC d_sharp{1.0f, 1.0f};
    if constexpr (TFAST && !SHARP1) d_sharp = make_divc(pr.bond_sharpness, ok);
    if constexpr (!kSplitTgtInAg<A, O, LPR> && !kSplitTgtInOb<A, O, LPR>)
        t.td = pair_dist<FAST>(ox, oy, tge[0], tge[1], ok);
#pragma unroll 64
    for (int i = 0; i < SP::NOB; ++i) {
        const int j = q + LPR * i;
        const bool valid = O % LPR == 0 || j < O;
        const bool tgt = kSplitTgtInOb<A, O, LPR> && i == SP::NOB - 1 && q == TQ;
        dst[i] = 0.0f;
        if (valid || tgt) {
            const float *pt = tgt ? tge : obe + 2 * (valid ? j : 0);
            const float d = pair_dist<FAST>(ox, oy, pt[0], pt[1], ok);
            dst[i] = d;
            if (valid) ob_min = __builtin_fminf(ob_min, d);
            else t.td = d;
        }
    }
#pragma unroll 64
    for (int i = 0; i < SP::NAG; ++i) {
        const int kx = q + LPR * i;
        const bool valid = (A - 1) % LPR == 0 || kx < A - 1;
        const bool tgt = kSplitTgtInAg<A, O, LPR> && i == SP::NAG - 1 && q == TQ;
        dst[SP::NOB + i] = 0.0f;
        if (valid || tgt) {
            const int m = valid ? kx + (kx >= a ? 1 : 0) : 0;
            const float *pt = tgt ? tge : sts + 5 * m;
            const float d = pair_dist<FAST>(ox, oy, pt[0], pt[1], ok);
            dst[SP::NOB + i] = d;
            if (!valid) {
                t.td = d;
            } else {
                ag_min = __builtin_fminf(ag_min, d);
                t.band += (pr.agents_min_d < d && d < pr.agents_max_d) ? 1 : 0;
                if constexpr (TFAST) {
                    const float sd = SHARP1 ? d - pr.ideal_dist : div_c(d - pr.ideal_dist, d_sharp, ok);
                    bond_row[kx] = recip_fast(1.0f + sd * sd, ok);
                } else {
                    const float sd = (d - pr.ideal_dist) / pr.bond_sharpness;
                    bond_row[kx] = 1.0f / (1.0f + sd * sd);
                }
            }
        }
    }
    t.fl |= (ob_min < pr.ob_risk_dist ? 1u : 0u) | (ob_min < pr.ob_coll_dist ? 2u : 0u) |
            (ag_min < pr.ag_risk_dist ? 4u : 0u) | (ag_min < pr.ag_coll_dist ? 8u : 0u);
    return t;
}

// Pass 2: the bearings of the pairs of split_dists (all of them, or with
// TGT_ONLY the target pair alone), written into the row as split_pairs
// writes them. Returns the target bearing on the lane that holds it.
template <int A, int O, int LPR, bool FAST, bool TGT_ONLY>
__device__ __forceinline__ float split_bearings(const float *__restrict__ sts,
                                                const float *__restrict__ obe,
                                                const float *__restrict__ tge, int a, int q,
                                                float ox, float oy, float dx, float dy,
                                                float *__restrict__ orow, float td,
                                                const MarlnavParams &pr, bool &ok,
                                                const float (&dst)[SplitSlots<A, O, LPR>::N])
{
    using SP = SplitPlan<A, O, LPR>;
    constexpr int TQ = LPR - 1;
    const float cap = pr.cap_distance;
    float ta = 0.0f;
    if constexpr (!kSplitTgtInAg<A, O, LPR> && !kSplitTgtInOb<A, O, LPR>) {
        ta = pair_angle<FAST>(ox, oy, tge[0], tge[1], dx, dy, td, cap, ok);
        if (q == 0) {
            orow[0] = ta;
            orow[1] = td;
        }
    }
#pragma unroll 64
    for (int i = 0; i < SP::NOB; ++i) {
        const int j = q + LPR * i;
        const bool valid = O % LPR == 0 || j < O;
        const bool tgt = kSplitTgtInOb<A, O, LPR> && i == SP::NOB - 1 && q == TQ;
        if ((valid && !TGT_ONLY) || tgt) {
            const float *pt = tgt ? tge : obe + 2 * (valid ? j : 0);
            const float ang = pair_angle<FAST>(ox, oy, pt[0], pt[1], dx, dy, dst[i], cap, ok);
            if (valid) {
                orow[2 + j] = ang;
                orow[2 + O + j] = dst[i];
            } else {
                orow[0] = ang;
                orow[1] = dst[i];
                ta = ang;
            }
        }
    }
#pragma unroll 64
    for (int i = 0; i < SP::NAG; ++i) {
        const int kx = q + LPR * i;
        const bool valid = (A - 1) % LPR == 0 || kx < A - 1;
        const bool tgt = kSplitTgtInAg<A, O, LPR> && i == SP::NAG - 1 && q == TQ;
        if ((valid && !TGT_ONLY) || tgt) {
            const int m = valid ? kx + (kx >= a ? 1 : 0) : 0;
            const float *pt = tgt ? tge : sts + 5 * m;
            const float ang =
                pair_angle<FAST>(ox, oy, pt[0], pt[1], dx, dy, dst[SP::NOB + i], cap, ok);
            if (!valid) {
                orow[0] = ang;
                orow[1] = dst[SP::NOB + i];
                ta = ang;
            } else {
                orow[2 + 2 * O + kx] = ang;
                orow[2 + 2 * O + (A - 1) + kx] = dst[SP::NOB + i];
            }
        }
    }
    return ta;
}

// The fresh env's row of agent a on this lane's slots (the native
// re-initialisation, environment.py:76-90, then observations() :105): the
// fresh agent (fx, fy, fdx, fdy) against the fresh obstacles `obf` (pair
// math, as reinit_reobs_tpl computes them), the target and other-agent slots
// from the formation's observation template `tv` (this lane's slots, loaded
// by the caller: raw bearing, distance; the cap applied here as in
// reobs_block_tpl).
template <int A, int O, int LPR, bool FAST>
__device__ __forceinline__ void split_fresh_row(const float *__restrict__ obf, int q, float fx,
                                                float fy, float fdx, float fdy,
                                                float *__restrict__ orow, float cap, bool &ok,
                                                const float2 (&tv)[SplitPlan<A, O, LPR>::NAG + 1])
{
    using SP = SplitPlan<A, O, LPR>;
    constexpr int TQ = LPR - 1;
    static_assert(kSplitTgtInAg<A, O, LPR>, "the target in the other-agent loop's spare slot");
#pragma unroll 64
    for (int i = 0; i < SP::NOB; ++i) {
        const int j = q + LPR * i;
        if (O % LPR == 0 || j < O) {
            const float px = obf[2 * j], py = obf[2 * j + 1];
            const float d = pair_dist<FAST>(fx, fy, px, py, ok);
            orow[2 + j] = pair_angle<FAST>(fx, fy, px, py, fdx, fdy, d, cap, ok);
            orow[2 + O + j] = d;
        }
    }
#pragma unroll
    for (int i = 0; i < SP::NAG; ++i) {
        const int kx = q + LPR * i;
        const bool valid = kx < A - 1;
        const bool tgt = i == SP::NAG - 1 && q == TQ;
        if (valid || tgt) {
            const float2 t = tv[i];
            const int sa = valid ? 2 + 2 * O + kx : 0;
            const int sd = valid ? 2 + 2 * O + (A - 1) + kx : 1;
            orow[sa] = t.y < cap ? 0.0f : t.x;  // the cap (environment.py:172-177)
            orow[sd] = t.y;
        }
    }
}

template <int A, int O, int LPR, bool OBS_ONLY, bool NOISY, bool OWN = false>
// (min 4 waves per SIMD: keeps the max-ilp scheduler (Makefile) within the
// 128 VGPRs of the 4-waves-per-SIMD grids; unbounded it takes 178 at A16/O32
// and halves occupancy)
__global__ void __launch_bounds__(64 * kWavesPerBlock, 4)
    split_kernel(float *h_states, const float *h_actions, const float *h_obstacles,
                 const float *h_target, const float *h_step_num, const uint8_t *h_terminates,
                 int64_t h_P, KArgs k)
{
    using SP = SplitPlan<A, O, LPR>;
    constexpr int EPW = SP::EPW, R = SP::R, D = SP::D;
    // the own-wave path stores raw row terms for wave 0's row_reward, which
    // wave 0 applies only when the row leaders do not (kSplitRRLeader)
    static_assert(!kSplitOwn<A, O, LPR, OWN> || !kSplitRRLeader<A, O>,
                  "kSplitOwn needs wave 0's row rewards (MARLNAV_SPLIT_RR_LEADER=0)");
    (void)k;  // read through kargs_late<kHotKargsOff>()
    extern __shared__ __attribute__((aligned(16))) float lds[];
#if MARLNAV_STAMPS
    int stamp_nfin = 0;
    int stamp_fast = 0;  // (the wave took the short pair math: bit 8 of the nfin slot)
#endif
#if MARLNAV_STAMPS
    unsigned long long t_entry;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_entry));
#endif
    const unsigned lane = threadIdx.x & 63;
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t gw = (int64_t)blockIdx.x * kWavesPerBlock + wib;
    const int64_t tile = gw;
    KArgsK *K = kargs_late<kHotKargsOff>();
    const int64_t P = h_P;
    if (tile * EPW >= P) return;  // (launch_split: ntiles = ceil(P / EPW) tiles)
    // the staging pointers come preloaded in SGPRs; the rest from KArgs
    StepPtrs b = load_ptrs(K);
    b.states = h_states;
    b.actions = h_actions;
    b.obstacles = const_cast<float *>(h_obstacles);
    b.target = const_cast<float *>(h_target);
    b.step_num = const_cast<float *>(h_step_num);
    b.terminates = const_cast<uint8_t *>(h_terminates);
    STAMP(0);
    if (MARLNAV_AB & 4096) return;  // (AB 4096: timing only - the launch alone)
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
    // kPre shapes (native re-init): the formation into FTP by LDS-DMA from
    // wave 0 (always live), with the tile's spans (the stage wait covers it),
    // for the fused re-init pass, whose pair items otherwise read it from
    // global memory after the per-env barrier
    constexpr bool kFormLds = kSplitSpread<A, O> && O <= 8 && MARLNAV_SPLIT_FORM_LDS && SP::NF <= 64;
    bool form_lds = false;
    if constexpr (kFormLds && !NOISY && !OBS_ONLY) {
        KArgsK *kl = kargs_late<kHotKargsOff>();
        const float *cfo = kl->a.b.formation;
        form_lds = cfo && !kl->a.b.fresh_states;
        if (form_lds && wib == 0 && lane < (unsigned)SP::NF)
            __builtin_amdgcn_global_load_lds(cfo + lane,
                                             (LdsVoid *)(lds + kWavesPerBlock * SP::FLOATS + SP::FTP),
                                             4, 0, 0);
    }
    const bool env_on = (int)lane < ne;
    float sn_in = 0.0f;
    unsigned term_in = 0u;
    if (!OBS_ONLY && env_on) {
        sn_in = b.step_num[e0 + lane];
        term_in = b.terminates[e0 + lane];
    }
    MarlnavParams pr = load_params(K);
    if constexpr (MARLNAV_OWN_VPIN == 2 || (MARLNAV_OWN_VPIN && kSplitOwn<A, O, LPR, OWN>)) {
        // the pair loops' and reward terms' parameters held in VGPRs: the
        // own-wave instantiation otherwise runs out of SGPRs (59 spilled to
        // VGPR lanes, reloaded in the observation's hot blocks; 20 left, in
        // cold blocks). Every split kernel (MARLNAV_OWN_VPIN 2): 4096x16x32
        // 11.23 -> 11.30 us, not taken
        const auto pin = [](float &x) { asm volatile("" : "+v"(x)); };
        pin(pr.ob_risk_dist); pin(pr.ob_coll_dist); pin(pr.ag_risk_dist); pin(pr.ag_coll_dist);
        pin(pr.agents_min_d); pin(pr.agents_max_d); pin(pr.ideal_dist); pin(pr.bond_sharpness);
        pin(pr.cap_distance); pin(pr.max_angle_diff); pin(pr.max_at_prop_d); pin(pr.init_dist);
        pin(pr.target_factor); pin(pr.heading_factor); pin(pr.distance_factor);
        pin(pr.soft_factor); pin(pr.bond_factor); pin(pr.risk_factor); pin(pr.target_radius);
        pin(pr.trunc_after);
    }
    const bool wt = (pr.flags & kWriteThroughFlag) != 0;  // written-through outputs
    float *const pre = lds + kWavesPerBlock * SP::FLOATS + SP::PRE;
    // the workgroup's live waves (the waves past the last tile have exited)
    const int64_t blk0 = (int64_t)blockIdx.x * kWavesPerBlock;
    const int live = (int)(K->a.ntiles - blk0 < kWavesPerBlock ? K->a.ntiles - blk0
                                                              : kWavesPerBlock);
    // (the fused native re-init of few-obstacle shapes only: at A16/O32 the
    // draws cost the stage ~1 us, more than they save in the tail)
    constexpr bool kPre = kSplitSpread<A, O> && O <= 8;
    if constexpr (kPre && !NOISY && !OBS_ONLY) {
        // native re-init: this wave's envs' fresh obstacles (Philox draws of
        // seed, step and env id), drawn while the staging loads are in
        // flight, so a finished env's workgroup-spread re-init reads them
        // instead of drawing after the per-env barrier
        KArgsK *kl = kargs_late<kHotKargsOff>();
        if (!kl->a.b.fresh_states) {
            const uint64_t sidx = kl->a.step_idx, g0 = (uint64_t)(kl->a.env_offset + e0);
#pragma unroll
            for (int k2 = 0; k2 * 64 < EPW * O; ++k2) {
                const int i = (int)lane + 64 * k2;
                const int cl = i % EPW, j = i / EPW;  // obstacle j of env cl
                if (((k2 + 1) * 64 <= EPW * O || i < EPW * O) && cl < ne) {
                    float v[2];
                    native_obst_draw(pr.seed, sidx, g0 + cl, j, pr.obs_range_x, pr.obs_mean_x,
                                     pr.obs_range_y, pr.obs_mean_y, v);
                    pre[(2 * j) * SP::EW + wib * EPW + cl] = v[0];
                    pre[(2 * j + 1) * SP::EW + wib * EPW + cl] = v[1];
                }
            }
        }
    }
    const int row = (int)lane / LPR, q = (int)lane - row * LPR;
    const int rowc = row < R ? row : 0;  // idle lanes shadow row 0 (results unused)
    const int el = rowc / A, a = rowc - el * A;
    const bool row_on = row < nr;
    unsigned c_trunc = 0, c_col = 0, c_tar = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS-DMA landed
    wave_sync();
    STAMP(1);
    if (MARLNAV_AB & 8192) return;  // (AB 8192: timing only - staged, then exit)

    // kSplitTpl (native re-init): the formation and its observation template
    // (NCP floats) into registers now, a few per thread, so their loads run
    // under the move and observe phases; every workgroup parks them in its
    // FTP region before the per-env barrier, for the one-pass re-init /
    // re-observation of finished envs (reinit_reobs_tpl). (Loaded after the
    // stage wait: no LDS-DMA is pending, so no LDS read waits for them.)
    constexpr int KCP = (SP::NCP + 64 * kWavesPerBlock - 1) / (64 * kWavesPerBlock);
    float cp[KCP];
    bool tpl_on = false;

    if constexpr (kSplitTpl<A, O> && !NOISY && !OBS_ONLY) {
        KArgsK *kl = kargs_late<kHotKargsOff>();
        const float *cfo = kl->a.b.formation, *ctp = kl->a.b.formation_obs;
        tpl_on = cfo && ctp && !kl->a.b.fresh_states;
        if (tpl_on) {
#pragma unroll
            for (int k2 = 0; k2 < KCP; ++k2) {
                const int idx = (int)threadIdx.x + k2 * 64 * kWavesPerBlock;
                if (idx < SP::NCP) cp[k2] = idx < SP::NF ? cfo[idx] : ctp[idx - SP::NF];
            }
        }
    }

    // ---- _move_agents (environment.py:113-123): every lane of a row moves
    // it (same instructions either way), the row leader stores it
    float ox = st[5 * rowc], oy = st[5 * rowc + 1];
    float dx = st[5 * rowc + 2], dy = st[5 * rowc + 3];
    if (!OBS_ONLY) {
        const float2 act = reinterpret_cast<const float2 *>(wl + SP::ACT)[rowc];
        float a0 = act.x, a1 = act.y;
        if (pr.flags & MARLNAV_SCALE_ACTIONS) {  // ActionScaler (utils.py:546-547)
            KArgsK *kl = kargs_late<kHotKargsOff>();
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

    // per-agent reward of a row (environment.py:184-234) from its reduced
    // terms: target bearing/distance, flags (1 ob_risk, 2 ob_col, 4 ag_risk,
    // 8 ag_col), in-band count and its A-1 bond terms (LDS):
    // (r_miss, r_hit, flags: 1 collision, 2 in target, 0)
    const auto row_reward = [&](float ta, float td, unsigned fl, int band,
                                const float *bond_row) -> float4 {
        const float head = fabsf(ta) < pr.max_angle_diff ? 1.0f : 0.0f;
        const float bandf = (float)band;
        const float bandc = bandf < pr.max_at_prop_d ? bandf : pr.max_at_prop_d;
        float bv[A - 1];
#pragma unroll
        for (int i = 0; i < A - 1; ++i) bv[i] = bond_row[i];
        const float bond = torch_row_sum_r<A - 1>(bv, [](float x) { return x; });
        const float dsc = bandc / pr.max_at_prop_d;
        const float soft = -1.0f * (td / pr.init_dist);
        const float bondm = bond / (float)(A - 1);
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
        const unsigned flags = ((fl & 10u) ? 1u : 0u) | ((td < pr.target_radius) ? 2u : 0u);
        return make_float4(rm, rh, __uint_as_float(flags), 0.0f);
    };

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
#if MARLNAV_STAMPS
        stamp_fast = fast ? 1 : 0;
#endif
        bool unused = true;
        SplitTerms t;
        if constexpr (kSplitOwn<A, O, LPR, OWN> && !OBS_ONLY) {
            // ---- kSplitOwn: distances first, the env's finished test, then
            // the bearings of the observation that stays (or of its target
            // pair alone) and, for a finished env, its fresh rows
            float dst[SplitSlots<A, O, LPR>::N];
            const bool tfast = (pr.flags & kTermsFastFlag) != 0;
            if (__builtin_expect(fast, 1) && tfast && pr.bond_sharpness == 1.0f)
                t = split_dists<A, O, LPR, true, true, true>(sts, obe, tge, a, q, ox, oy, brow, pr,
                                                            unused, dst);
            else if (__builtin_expect(fast, 1) && tfast)
                t = split_dists<A, O, LPR, true, true, false>(sts, obe, tge, a, q, ox, oy, brow, pr,
                                                             unused, dst);
            else if (__builtin_expect(fast, 1))
                t = split_dists<A, O, LPR, true, false, false>(sts, obe, tge, a, q, ox, oy, brow,
                                                              pr, unused, dst);
            else
                t = split_dists<A, O, LPR, false, false, false>(sts, obe, tge, a, q, ox, oy, brow,
                                                               pr, unused, dst);
            const unsigned fl = lpr_or<LPR>(t.fl);
            const int band = lpr_sum<LPR>(t.band);
            // per_env's test (environment.py:96-104, 213-214) on the wave's env:
            // its step number and `terminates` on lane 0, its rows' collisions
            const float sn0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sn_in), 0));
            const unsigned tm0 = (unsigned)__builtin_amdgcn_readlane((int)term_in, 0);
            const bool col = __ballot(row_on && (fl & 10u) != 0u) != 0ull;
            const bool own_fin = tpl_on && !(MARLNAV_AB & 1) &&
                                 (sn0 + 1.0f > pr.trunc_after || tm0 != 0u || col);
            if (!own_fin) {
                if (__builtin_expect(fast, 1))
                    split_bearings<A, O, LPR, true, false>(sts, obe, tge, a, q, ox, oy, dx, dy, orow,
                                                           t.td, pr, unused, dst);
                else
                    split_bearings<A, O, LPR, false, false>(sts, obe, tge, a, q, ox, oy, dx, dy,
                                                            orow, t.td, pr, unused, dst);
            } else {
                if (__builtin_expect(fast, 1))
                    split_bearings<A, O, LPR, true, true>(sts, obe, tge, a, q, ox, oy, dx, dy, orow,
                                                          t.td, pr, unused, dst);
                else
                    split_bearings<A, O, LPR, false, true>(sts, obe, tge, a, q, ox, oy, dx, dy,
                                                           orow, t.td, pr, unused, dst);
            }
            wave_sync();  // bond terms and the target pair of each row are in LDS
            if (row_on && q == 0) {
                t.ta = orow[0];  // computed by lane LPR-1
                t.td = orow[1];
                reinterpret_cast<float4 *>(wl + SP::RED)[row] =
                    make_float4(t.ta, t.td, __uint_as_float(fl), __int_as_float(band));
            }
            if (own_fin) {
                // ---- the fresh env (environment.py:76-90, 104-105) on this
                // wave: blends of the state and target, the fresh obstacles
                // (one Philox block per obstacle lane), then its rows - the
                // formation template's target / other-agent pairs and the
                // obstacle pairs, or every pair computed when a blend left the
                // formation's bits (a non-finite old value)
                wave_sync();  // the row leaders have read the old target pair
                KArgsK *kl = kargs_late<kHotKargsOff>();
                const float *form = kl->a.b.formation;
                const float2 *tpg = reinterpret_cast<const float2 *>(kl->a.b.formation_obs);
                float2 tv[SplitPlan<A, O, LPR>::NAG + 1];
#pragma unroll
                for (int i = 0; i < SplitPlan<A, O, LPR>::NAG; ++i) {  // (loads first)
                    const int kx = q + LPR * i;
                    const bool valid = kx < A - 1;
                    const bool tgt = i == SplitPlan<A, O, LPR>::NAG - 1 && q == LPR - 1;
                    tv[i] = (valid || tgt) ? tpg[rowc * A + (valid ? kx + 1 : 0)] : make_float2(0.f, 0.f);
                }
                tv[SplitPlan<A, O, LPR>::NAG] = make_float2(0.f, 0.f);
                const SplitEnvs<A, O, EPW, SP::FLOATS, SP::ST, SP::OB, SP::TG, SP::OBS, SP::DP> ev{
                    lds, blk0 * EPW};
                const int c = wib * EPW;
                const int64_t e = ev.env(c);
                bool uncl = false;
                for (int k2 = (int)lane; k2 < 5 * A + 2; k2 += 64) {
                    const bool tg = k2 >= 5 * A;
                    float *d = tg ? ev.targ(c) + (k2 - 5 * A) : ev.state(c) + k2;
                    const float vb = blend_in(*d, form[k2]);
                    *d = vb;
                    if (tg) out_el(kl->a.b.target, 2 * e + (k2 - 5 * A), vb);
                    uncl |= (tg || k2 % 5 < 4) && __float_as_uint(vb) != __float_as_uint(form[k2]);
                }
                for (int j = (int)lane; j < O; j += 64) {
                    float v[2];
                    native_obst_draw(kl->p.seed, kl->a.step_idx, (uint64_t)(kl->a.env_offset + e),
                                     j, kl->p.obs_range_x, kl->p.obs_mean_x, kl->p.obs_range_y,
                                     kl->p.obs_mean_y, v);
                    float *o = ev.obst(c) + 2 * j;
                    o[0] = blend_in(o[0], v[0]);
                    o[1] = blend_in(o[1], v[1]);
                    out_el(kl->a.b.obstacles, e * O * 2 + 2 * j, o[0]);
                    out_el(kl->a.b.obstacles, e * O * 2 + 2 * j + 1, o[1]);
                }
                wave_sync();
                if (__ballot(uncl) == 0ull) {
                    const float *fs = st + 5 * rowc;  // the blended (= formation) agent row
                    const float fx = fs[0], fy = fs[1], fdx = fs[2], fdy = fs[3];
                    const bool cok2 = coord_ok(fx) && coord_ok(fy) &&
                                      tile_coords_ok<EPW * O * 2, 0>(wl + SP::OB, wl + SP::TG, lane);
                    if (__ballot(!cok2) == 0ull)
                        split_fresh_row<A, O, LPR, true>(wl + SP::OB, q, fx, fy, fdx, fdy, orow,
                                                         pr.cap_distance, unused, tv);
                    else
                        split_fresh_row<A, O, LPR, false>(wl + SP::OB, q, fx, fy, fdx, fdy, orow,
                                                          pr.cap_distance, unused, tv);
                } else {
                    reobs_block<A, O>(ev, OneEnv{c}, 1, pr.cap_distance, (int)lane, 64);
                }
            }
        } else if (__builtin_expect(fast, 1) && !OBS_ONLY && (pr.flags & kTermsFastFlag) &&
            pr.bond_sharpness == 1.0f)
            t = split_pairs<A, O, LPR, !OBS_ONLY, true, true, true>(sts, obe, tge, a, q, ox, oy, dx,
                                                                   dy, orow, brow, pr, unused);
        else if (__builtin_expect(fast, 1) && !OBS_ONLY && (pr.flags & kTermsFastFlag))
            t = split_pairs<A, O, LPR, !OBS_ONLY, true, true>(sts, obe, tge, a, q, ox, oy, dx, dy,
                                                             orow, brow, pr, unused);
        else if (__builtin_expect(fast, 1))
            t = split_pairs<A, O, LPR, !OBS_ONLY, true>(sts, obe, tge, a, q, ox, oy, dx, dy, orow,
                                                       brow, pr, unused);
        else
            t = split_pairs<A, O, LPR, !OBS_ONLY, false>(sts, obe, tge, a, q, ox, oy, dx, dy, orow,
                                                        brow, pr, unused);
        if (!OBS_ONLY && !kSplitOwn<A, O, LPR, OWN>) {
            const unsigned fl = lpr_or<LPR>(t.fl);
            const int band = lpr_sum<LPR>(t.band);
            wave_sync();  // bond terms of the row are in LDS
            if (row_on && q == 0) {
                if constexpr (kSplitTgtInAg<A, O, LPR> || kSplitTgtInOb<A, O, LPR>) {
                    t.ta = orow[0];  // computed by lane LPR-1 (wave_sync above)
                    t.td = orow[1];
                }
                if constexpr (kSplitSpread<A, O> && !kSplitRRLeader<A, O>) {
                    // the row's reduced terms; wave 0 finishes every row of
                    // the workgroup after the barrier (row_reward)
                    reinterpret_cast<float4 *>(wl + SP::RED)[row] =
                        make_float4(t.ta, t.td, __uint_as_float(fl), __int_as_float(band));
                } else {
                    reinterpret_cast<float4 *>(wl + SP::RED)[row] =
                        row_reward(t.ta, t.td, fl, band, brow);
                }
            }
        }
    }
    STAMP(3);

    // ---- the tile's rows and states from LDS to global memory (the end of
    // the step)
    const auto store_tile = [&]() {
        {
            const float *src = wl + SP::OBS;
            float *gobs = in_sgpr(b.obs + e0 * (A * D));
            const int n = nr * D;
            constexpr int VAL = gcd_c(R * D * 4, 16);  // tile base alignment in bytes
            float *gnorm = nullptr;
            const float *mean = nullptr, *scale = nullptr;
            if (!OBS_ONLY && (pr.flags & MARLNAV_WRITE_OBS_NORM)) {
                KArgsK *kl = kargs_late<kHotKargsOff>();
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
                        // (AB 2048: timing only - consecutive pieces, no bank
                        // conflicts: the most an XOR swizzle of the pieces can save)
                        const float4 v = *reinterpret_cast<const float4 *>(
                            (MARLNAV_AB & 2048) ? src + 4 * i : src + rr * SP::DP + 4 * c4);
                        if (kWtOut && wt)
                            wt_st4(out_buf(gobs, 4u * n), 16u * i, v);
                        else
                            out_st4<kNtRows>(gobs + 4 * i, v);
                    }
                } else {
                    for (int i = (int)lane; i < n; i += 64) {
                        const int rr = i / D;
                        const float v = src[rr * SP::DP + (i - rr * D)];
                        if (kWtOut && wt)
                            wt_st(out_buf(gobs, 4u * n), 4u * i, v);
                        else
                            out_st<kNtRows>(gobs + i, v);
                    }
                }
            } else if (VAL % 16 == 0 && ne == EPW) {
                for (int i = (int)lane; i < n / 4; i += 64) {
                    const float4 v = reinterpret_cast<const float4 *>(src)[i];
                    if (kWtOut && wt)
                        wt_st4(out_buf(gobs, 4u * n), 16u * i, v);
                    else
                        out_st4<kNtRows>(gobs + 4 * i, v);
                }
            } else if (VAL % 8 == 0 && n % 2 == 0) {
                for (int i = (int)lane; i < n / 2; i += 64) {
                    const float2 v = reinterpret_cast<const float2 *>(src)[i];
                    if (kWtOut && wt)
                        wt_st2(out_buf(gobs, 4u * n), 8u * i, v);
                    else
                        out_st2<kNtRows>(gobs + 2 * i, v);
                }
            } else {
                for (int i = (int)lane; i < n; i += 64) {
                    if (kWtOut && wt)
                        wt_st(out_buf(gobs, 4u * n), 4u * i, src[i]);
                    else
                        out_st<kNtRows>(gobs + i, src[i]);
                }
            }
            if (gnorm) {
                const OutBuf nb = out_buf(gnorm, 4u * n);
    #pragma unroll 8  // (mean/scale loads of 8 iterations in flight at once)
                for (int i = (int)lane; i < n; i += 64) {
                    const int rr = i / D, kk = i - rr * D;
                    const float v = (src[rr * SP::DP + kk] - mean[kk]) / scale[kk];
                    if (kWtOut && wt)
                        wt_st(nb, 4u * i, v);
                    else
                        gnorm[i] = v;
                }
            }
        }
        if (!OBS_ONLY) {
            float *gst = in_sgpr(b.states_out + e0 * (A * 5));
            const int n = nr * 5;
            constexpr int SAL = gcd_c(R * 20, 16);
            if (SAL % 16 == 0 && ne == EPW) {
                for (int i = (int)lane; i < n / 4; i += 64) {
                    const float4 v = reinterpret_cast<const float4 *>(st)[i];
                    if (kWtOut && wt)
                        wt_st4(out_buf(gst, 4u * n), 16u * i, v);
                    else
                        out_st4<kNtRows>(gst + 4 * i, v);
                }
            } else {
                for (int i = (int)lane; i < n; i += 64) {
                    if (kWtOut && wt)
                        wt_st(out_buf(gst, 4u * n), 4u * i, st[i]);
                    else
                        out_st<kNtRows>(gst + i, st[i]);
                }
            }
        }
    };

    bool stored = false;  // (the tile went out before the per-env barrier)
    bool tail_wg = false;  // (AB 1 << 19, timing only: a workgroup with finished envs skips its stores)
    if (!OBS_ONLY) {
        wave_sync();
        // ---- per-env reductions, terminal logic, masked re-init (env e,
        // reward rows `red` (A float4: r_miss, r_hit, flags), step number and
        // `terminates` in); returns fin and sets the counter flags
        bool tr_l = false, co_l = false, ta_l = false;
        const auto per_env = [&](int64_t e, const float4 *red, float sn_v, unsigned term_v,
                                 float *s5, float *obl, float *tgl) -> bool {
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
            const auto put_f = [&](float *arr, float v) { out_el(arr, e, v); };
            const auto put_b = [&](uint8_t *arr, uint8_t v) { out_el(arr, e, v); };
            put_f(b.reward, rsum / (float)A);                  // torch.mean (:233)
            float step_num = sn_v + 1.0f;                      // :96
            const bool truncated = step_num > pr.trunc_after;  // :97
            const bool term_old = term_v != 0u;
            const bool terminated = any_col || term_old;       // :213-214
            put_b(b.terminates, (uint8_t)(!term_old && all_in));  // :218-219
            put_b(b.terminated, (uint8_t)terminated);
            put_b(b.truncated, (uint8_t)truncated);
            const bool fin = truncated || terminated;          // :102-104
            if (fin && (NOISY || !kSplitSpread<A, O>)) {  // per-env re-init on the env lane
                KArgsK *kl = kargs_late<kHotKargsOff>();
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
                for (int i = 0; i < 2 * O; ++i) out_el(gob, e * O * 2 + i, obl[i]);
                out_el(gtg, 2 * e, tgl[0]);
                out_el(gtg, 2 * e + 1, tgl[1]);
            }
            if (fin) step_num = blend_in(step_num, 0.0f);
            put_f(b.step_num, step_num);
            tr_l = truncated;
            co_l = any_col;
            ta_l = all_in;
            return fin;
        };

        if constexpr (kSplitSpread<A, O>) {
            // ---- the workgroup's finished envs, re-initialised (:104) and
            // re-observed (:105) by all its threads: a finished env costs its
            // wave ~1/4 of a full observation pass instead of a second pass
            // on its own lanes (the straggler that set the kernel's end).
            // The per-env phase of all the workgroup's envs runs on wave 0
            // (one lane per env) after one barrier, instead of on one or two
            // lanes of every wave: the other waves' VALU is not spent on it.
            int *bcnt = reinterpret_cast<int *>(lds + kWavesPerBlock * SP::FLOATS);
            int *bslot = bcnt + kWavesPerBlock;
            int *unclean = bslot + kWavesPerBlock * EPW;
            float *bsn = reinterpret_cast<float *>(bcnt) + SP::ENVIN;
            unsigned *bterm = reinterpret_cast<unsigned *>(bsn + kWavesPerBlock * EPW);
            if (threadIdx.x == 0) *unclean = 0;
            if (tpl_on) {  // (uniform: every wave holds its part)
                float *ftp = lds + kWavesPerBlock * SP::FLOATS + SP::FTP;
#pragma unroll
                for (int k2 = 0; k2 < KCP; ++k2) {
                    const int idx = (int)threadIdx.x + k2 * 64 * kWavesPerBlock;
                    if (idx < SP::NCP) ftp[idx] = cp[k2];
                }
            }
            if (env_on) {
                bsn[wib * EPW + (int)lane] = sn_in;
                bterm[wib * EPW + (int)lane] = term_in;
            }
            if constexpr (MARLNAV_SPLIT_EARLY && kSplitOwn<A, O, LPR, OWN>) {
                // own-wave re-init: the tile (rows and states) is final here,
                // so it streams out under wave 0's per-env phase
                if (tpl_on && !(MARLNAV_AB & 2)) {
                    wave_sync();
                    store_tile();
                    stored = true;
                }
            }
            __syncthreads();
            STAMP(4);
            if (MARLNAV_AB & 16384) return;  // (AB 16384: timing only - observed, then exit)
            if (wib == 0) {
                if (MARLNAV_SPLIT_PRIO) __builtin_amdgcn_s_setprio(MARLNAV_SPLIT_PRIO);  // (A/B builds)
                // every row of the workgroup: its reward terms (one lane per
                // row, all 64 lanes busy where the row leaders were 1 in LPR)
                static_assert(kWavesPerBlock * R <= 64, "one lane per row of the workgroup");
                if (!kSplitRRLeader<A, O> && (int)lane < live * R) {
                    const int cw = (int)lane / R, rw = (int)lane - cw * R;
                    float *wlc = lds + cw * SP::FLOATS;
                    float4 *rp = reinterpret_cast<float4 *>(wlc + SP::RED) + rw;
                    const float4 tv = *rp;
                    if ((blk0 + cw) * EPW + rw / A < P)
                        *rp = row_reward(tv.x, tv.y, __float_as_uint(tv.z), __float_as_int(tv.w),
                                         wlc + SP::BOND + rw * (A - 1));
                }
                wave_sync();
                STAMPX(0);
                const int ce = (int)lane;  // env code: wave ce / EPW, env ce % EPW
                const int64_t e = blk0 * EPW + ce;
                const bool on = ce < live * EPW && e < P;
                bool fin = false;
                if (on) {
                    const int cw = ce / EPW, cl = ce - cw * EPW;
                    float *wlc = lds + cw * SP::FLOATS;
                    fin = per_env(e, reinterpret_cast<const float4 *>(wlc + SP::RED) + A * cl,
                                  bsn[ce], bterm[ce], wlc + SP::ST + 5 * A * cl,
                                  wlc + SP::OB + 2 * O * cl, wlc + SP::TG + 2 * cl);
                }
                const uint64_t fm = __ballot(fin);
                if (fin)
                    bslot[__builtin_amdgcn_mbcnt_hi((unsigned)(fm >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((unsigned)fm, 0u))] = ce;
                if (lane == 0) bcnt[0] = (int)__popcll(fm);
                c_trunc = __popcll(__ballot(tr_l));
                c_col = __popcll(__ballot(co_l));
                c_tar = __popcll(__ballot(ta_l));
                STAMPX(1);
                if (MARLNAV_SPLIT_PRIO) __builtin_amdgcn_s_setprio(0);
            }
            __syncthreads();
            STAMPX(2);
            if (MARLNAV_AB & 32768) return;  // (AB 32768: timing only - per-env done, then exit)
            const FlatFinList list{bslot, bcnt[0]};
#if MARLNAV_STAMPS
            stamp_nfin = list.total();
            for (int f = 0; f < list.total(); ++f)  // (bit 9: this wave's own env finished)
                if (list[f] / EPW == wib) stamp_nfin |= 1 << 9;
#endif
            // (kSplitOwn with the template: every finished env was re-initialised
            // and re-observed by its own wave before the per-env barrier)
            const bool own_done = kSplitOwn<A, O, LPR, OWN> && tpl_on;
            if ((MARLNAV_AB & (1 << 19)) && list.total()) tail_wg = true;
            if (const int nfin = ((MARLNAV_AB & 1) || own_done) ? 0 : list.total()) {  // (AB 1: timing only)
                KArgsK *kl = kargs_late<kHotKargsOff>();
                const SplitEnvs<A, O, EPW, SP::FLOATS, SP::ST, SP::OB, SP::TG, SP::OBS, SP::DP> ev{
                    lds, blk0 * EPW};
                // waves past the last tile have exited: items go to the live ones
                const int tid = (int)threadIdx.x, nt = 64 * live;
                // fused native re-init + re-observation recomputes a Philox
                // block per obstacle pair: only for few obstacles
                if (!NOISY && O <= 8 && !kl->a.b.fresh_states) {
                    const float *form = form_lds ? lds + kWavesPerBlock * SP::FLOATS + SP::FTP
                                                 : kl->a.b.formation;
                    reinit_reobs_native<A, O, SP::EW>(kl, ev, form, list, nfin,
                                                      pr.cap_distance, tid, nt, pre);
                    __syncthreads();
                } else if (kSplitTplPass<A, O> && tpl_on && live == kWavesPerBlock) {
                    if constexpr (kSplitTplPass<A, O>) {
                        // one pass (formation and template parked by every wave)
                        const float *ftp = lds + kWavesPerBlock * SP::FLOATS + SP::FTP;
                        reinit_reobs_tpl<A, O, 64 * kWavesPerBlock>(
                            kl, ev, ftp, reinterpret_cast<const float2 *>(ftp + SP::NF), list,
                            nfin, pr.cap_distance, tid, unclean);
                        __syncthreads();
                        STAMPX(3);
                        if (*unclean) {  // an agent or target off the formation: every pair
                            reobs_block<A, O>(ev, list, nfin, pr.cap_distance, tid, nt);
                            __syncthreads();
                        }
                    }
                } else {
                    if (!NOISY) {
                        reinit_block<A, O, kPre ? SP::EW : 0>(
                            kl, ev, kl->a.b.formation, list, nfin, tid, nt, nullptr, pre);
                        __syncthreads();
                    }
                    reobs_block<A, O>(ev, list, nfin, pr.cap_distance, tid, nt);
                    __syncthreads();
                }
            }
        } else {
            bool fin = false;
            if (env_on)
                fin = per_env(e0 + lane, reinterpret_cast<const float4 *>(wl + SP::RED) + A * lane,
                              sn_in, term_in, st + 5 * A * lane, wl + SP::OB + 2 * O * lane,
                              wl + SP::TG + 2 * lane);
            const uint64_t finmask = __ballot(fin);
            c_trunc = __popcll(__ballot(tr_l));
            c_col = __popcll(__ballot(co_l));
            c_tar = __popcll(__ballot(ta_l));
            STAMP(4);
            if (finmask) {
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
    }
    STAMP(5);

    // ---- stream the tile out (obs rows and states from LDS)
    wave_sync();
    if (MARLNAV_AB & 2) return;  // (AB 2: timing only - no store)
    if ((MARLNAV_AB & (1 << 19)) && tail_wg) return;
    if (!stored) store_tile();
    STAMP(6);
    if (!OBS_ONLY && lane == 0 && (c_trunc | c_col | c_tar)) {
        KArgsK *kl = kargs_late<kHotKargsOff>();
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
        *STAMP_PTR((size_t)gw * 24 + 16) = t_entry;
        *STAMP_PTR((size_t)gw * 24 + 17) = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        *STAMP_PTR((size_t)gw * 24 + 18) = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
        *STAMP_PTR((size_t)gw * 24 + 19) = (unsigned)stamp_nfin | ((unsigned)stamp_fast << 8);
    }
#endif
}
