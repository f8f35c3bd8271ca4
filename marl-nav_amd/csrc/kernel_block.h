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
template <int A, int O>
struct BlockPlan {
    static constexpr int E = 64, R = E * A, D = 2 + 2 * O + 2 * (A - 1);
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
    static constexpr int FLOATS = FRESH + 2 * O * E;
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
template <int A, int O>
struct BlockSpans {
    using BP = BlockPlan<A, O>;
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

// The end-of-step state of one env (environment.py:96-97 step count and
// truncation, :213-219 collision / target flags, :102-104 finished) from its
// agents' row flags (RowOut.flags: bit0 collision, bit1 in target) and its
// staged step_num / terminates. The one definition of "finished": wave 0's
// per-env phase (its outputs) and waves 1..A-1 (the re-init set and the
// early-store decision) both evaluate it on the same LDS inputs, so the two
// finished sets cannot drift apart.
struct EnvEnd {
    unsigned any_col, all_in;
    float step_num;  // incremented (:96)
    bool truncated, term_old, terminated, fin;
};

// flag(i): agent i's RowOut.flags word
template <int A, class F>
__device__ __forceinline__ EnvEnd env_end(F flag, float step_num_old, uint8_t terminates_old,
                                          float trunc_after)
{
    EnvEnd e;
    e.any_col = 0u;
    e.all_in = 1u;
#pragma unroll
    for (int i = 0; i < A; ++i) {
        const unsigned f = flag(i);
        e.any_col |= f & 1u;
        e.all_in &= (f >> 1) & 1u;
    }
    e.step_num = step_num_old + 1.0f;             // :96
    e.truncated = e.step_num > trunc_after;       // :97
    e.term_old = terminates_old != 0;
    e.terminated = e.any_col != 0u || e.term_old;  // :213-214
    e.fin = e.truncated || e.terminated;          // :102-104
    return e;
}

// Where a block with no finished env stores its rows and states: under the
// per-env phase, from waves 1..A-1 (true), or after the last barrier. The
// stores hold their waves at issue until the HBM-bound write burst drains
// (DESIGN.md §5 "Where the stores go"): that pays where the observe phase is
// long against the burst and loses at A3/O3 (graph replay, early vs after,
// profiles/r04_ab_early_out.txt: 65536x3x8 10.54 -> 9.81 us, 131072x3x8
// 18.10 -> 17.44, 32768x3x8 8.19 -> 8.07; 65536x3x3 6.98 -> 7.13, 16384x3x3
// 5.18 -> 5.29, 131072x3x3 11.43 -> 11.53). Round 6, final kernels, re-measured
// at A3/O3 (profiles/r06_ab_revalidate.txt, four runs on three boxes, graph
// replay and stream launches): 65536x3x3 -0.03 to -0.04 us, 131072x3x3 -0.10 to
// -0.15, 32768x3x3 +0.01, but the draw-wave instantiation (16384x3x3, one
// block per CU) +0.08: so every instantiation but the draw-wave one.
// MARLNAV_EARLY_OUT 0 / 1 forces it (A/B builds).
template <int A, int O, bool HELP>
constexpr bool kBlockEarlyOut = MARLNAV_EARLY_OUT < 0 ? (O >= 8 || !HELP) : MARLNAV_EARLY_OUT != 0;

// Phases (one block barrier after each of the first four): stage | move +
// coordinate check | observe into LDS rows | per-env phase on wave 0 while
// waves 1..A-1 re-initialise and re-observe the finished envs (native
// re-init; none in most blocks) | rows and states stream out of LDS.
// (Two blocks per workgroup, software-pipelined - tile 1's loads under tile
// 0's compute, tile 0's stores under tile 1's - measured bit-exact and
// slower, 65536x3x3 6.44 -> 9.45 us: profiles/r06_ab_pipe.txt, code at
// 16437ed.)
template <int A, int O, bool OBS_ONLY, bool NOISY, bool HELP = false>
__global__ void __launch_bounds__(64 * (A + HELP))
    block_kernel(float *h_states, const float *h_actions, const float *h_obstacles,
                 const float *h_target, const float *h_step_num, const uint8_t *h_terminates,
                 int64_t h_P, KArgs k)
{
    using BP = BlockPlan<A, O>;
    // NT: the agent waves' threads, over which every work loop is spread
    // (HELP: one more wave, w == A, draws the fresh obstacles and otherwise
    // only meets the barriers)
    constexpr int E = BP::E, R = BP::R, D = BP::D, NT = BP::NT;
    static_assert(!HELP || (!OBS_ONLY && !NOISY), "the draw wave serves the native re-init step");
    (void)k;  // read through kargs_late<kHotKargsOff>()
    extern __shared__ __attribute__((aligned(16))) float lds[];
#if MARLNAV_STAMPS
    unsigned long long t_entry;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_entry));
#endif
    if (MARLNAV_AB & 4096) return;  // (AB 4096: timing only - the launch alone)
    const int tid = (int)threadIdx.x;
    const unsigned lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // agent of this wave
    const bool hw = HELP && w == A;  // the draw wave (no agent)
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
    using BS = BlockSpans<A, O>;
    // The block's phases are the body of a lambda called once: this form
    // gives block_kernel<3,3> 87 VGPRs and no SGPR spill lanes where the
    // plain body had 88 and 4 (65536x3x3 6.53 -> 6.44 us steady, 32768x3x3
    // 5.30 -> 5.23, same box: profiles/r06_ab_pipe.txt)
    auto block = [&]() __attribute__((always_inline)) {
    const int64_t blk = blockIdx.x;
    const int64_t gw = blk * (A + HELP) + w;  // stamps slot
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
    float *actw = lds + BP::ACTW + 2 * E * (hw ? 0 : w);  // x at [l], y at [E + l]
    if (!OBS_ONLY && full && !hw) {
        const float *pa = h_actions + ((e0 + lane) * A + w) * 2;
        __builtin_amdgcn_global_load_lds(pa, (LdsVoid *)actw, 4, 0, 0);
        __builtin_amdgcn_global_load_lds(pa + 1, (LdsVoid *)(actw + E), 4, 0, 0);
    }
    // ---- stage the block (spans spread over the waves: span k by wave k % A)
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
    } else if (!hw) {
        const int nr = ne * A;
        block_copy(b.states + e0 * (A * 5), st, nr * 5, tid, NT);
        if (!OBS_ONLY && (int)lane < ne) {  // (each lane its own slots: no barrier)
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
    // (one Philox block per thread at most: O <= A. At A3/O8 the draws go
    // to the finished-env tail instead: three blocks per thread here cost
    // the stage phase more than they save there, 131072x3x8 18.4 -> 19.0 us
    // with the round-4 Philox4x32)
    constexpr bool kPre = E * O <= NT;
    if constexpr (HELP) {
        // the draw wave: the same draws, O per lane (env `lane`), on the
        // SIMD the agent waves leave idle
        if (hw && overlap && !(MARLNAV_AB & 256) && (int)lane < ne) {
            KArgsK *kl = kargs_late<kHotKargsOff>();
            const uint64_t sidx = kl->a.step_idx, g = (uint64_t)(kl->a.env_offset + e0) + lane;
            float *pre = lds + BP::FRESH;
            float v[O][2];
#pragma unroll
            for (int j = 0; j < O; ++j)
                native_obst_draw(pr.seed, sidx, g, j, pr.obs_range_x, pr.obs_mean_x, pr.obs_range_y,
                                 pr.obs_mean_y, v[j]);
#pragma unroll
            for (int j = 0; j < O; ++j) {
                pre[(2 * j) * E + lane] = v[j][0];
                pre[(2 * j + 1) * E + lane] = v[j][1];
            }
        }
    } else if (kPre && overlap && !(MARLNAV_AB & 256)) {  // (AB 256: timing only, no draws)
        // the fresh obstacles of every env of the block (its Philox draws
        // depend only on seed, step and env id), drawn while the staging
        // loads are in flight: a finished env's re-init then reads them
        // instead of drawing after the per-env barrier, where the draws sat
        // on the block's critical path (65536x3x3: 0.25 us of 0.63). Item
        // i = obstacle i / E of env i % E: at E = 64 the obstacle index is
        // the wave's, so the Philox key is wave-uniform (SALU).
        KArgsK *kl = kargs_late<kHotKargsOff>();
        const uint64_t sidx = kl->a.step_idx, g0 = (uint64_t)(kl->a.env_offset + e0);
        float *pre = lds + BP::FRESH;
#pragma unroll
        for (int k2 = 0; k2 * NT < E * O; ++k2) {
            const int i = tid + k2 * NT;
            const int l = i % E, j = __builtin_amdgcn_readfirstlane(i / E);
            if (((k2 + 1) * NT <= E * O || i < E * O) && l < ne) {
                float v[2];
                native_obst_draw(pr.seed, sidx, g0 + l, j, pr.obs_range_x, pr.obs_mean_x,
                                 pr.obs_range_y, pr.obs_mean_y, v);
                pre[(2 * j) * E + l] = v[0];
                pre[(2 * j + 1) * E + l] = v[1];
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
        float a0 = actw[lane];
        a1 = actw[E + lane];
        STAMPS_S(0);  // (substamps: this wave's actions landed)
        if (pr.flags & MARLNAV_SCALE_ACTIONS) {  // ActionScaler (utils.py:546-547)
            KArgsK *kl = kargs_late<kHotKargsOff>();
            a0 = kl->p.act_scale[0] * a0 + kl->p.act_mean[0];
            a1 = kl->p.act_scale[1] * a1 + kl->p.act_mean[1];
        }
        sincos_k(clamp_t(a0, -kPiF, kPiF), &sn, &c);
#if MARLNAV_STAMPS && MARLNAV_SUBSTAMPS
        asm volatile("" ::"v"(sn), "v"(c));
#endif
        STAMPS_S(1);  // (substamps: the heading's sin/cos done)
    }
    const int l = (int)lane;  // env of this lane within the block
    const int r = l * A + (hw ? 0 : w);  // row of this lane (the draw wave has none)
    const bool row_on = l < ne && !hw;
    const int nrow = ne * A;
    int *bad_word = reinterpret_cast<int *>(lds + BP::FLG) + 1;  // any coordinate off the fast range
    if (tid == 0) *bad_word = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA landed
    STAMPS_S(2);  // (substamps: every span this wave issued landed)
    __syncthreads();
    STAMP(1);
    if (MARLNAV_AB & 8192) {  // (AB 8192: timing / census only - staged, then exit;
        asm volatile("" ::"v"(sn), "v"(c), "v"(a1));  // the sin/cos kept alive)
        return;
    }

    // obstacle and target coordinates of the block for the pair-math choice
    // (below); read before the move writes LDS, so the reads overlap it
    // (a partial last block takes the IEEE path without checking)
    CoordRange crange;
    if (full && !hw) {
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
    if (full && !hw) {
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
    const bool fast = full && *bad_word == 0;

    // ---- observations of the moved state + reward terms (:99-100)
    float4 *red = reinterpret_cast<float4 *>(lds + BP::RED);
    float *obs_rows = lds + BP::OBS;
    if (row_on) {
        float rowv[D];
        RowOut ro;
        bool unused = true;
        if (__builtin_expect(fast, 1) && !MARLNAV_AB_NOREFC && pr.bond_sharpness == 1.0f &&
            pr.max_at_prop_d == 2.0f)
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
#if MARLNAV_STAMPS && MARLNAV_SUBSTAMPS
        asm volatile("" ::"v"(ro.r_miss), "v"(rowv[0]), "v"(rowv[D - 1]));
#endif
        STAMPS_S(3);  // (substamps: this lane's row computed)
        lds_row_write<D>(obs_rows + r * D, rowv);
        if (!OBS_ONLY) red[r] = make_float4(ro.r_miss, ro.r_hit, __uint_as_float(ro.flags), 0.0f);
    }
    __syncthreads();
    STAMP(3);
    if (MARLNAV_AB & 16384) return;  // (AB 16384: timing only - observed, then exit)
    // the output pointers, read again from the kernarg segment here: no
    // scalar register holds them through the observation, where the entry
    // copies spilled 14 SGPRs to VGPR lanes (65536x3x3 6.55 -> 6.33 us,
    // profiles/r05_ab_late_ptrs.txt; MARLNAV_LATE_PTRS=0: the entry copies)
    StepPtrs bo;
    if constexpr (MARLNAV_LATE_PTRS) bo = load_ptrs(kargs_late<kHotKargsOff>());
    else bo = b;
    float *gobs = in_sgpr(bo.obs + e0 * (A * D));
    if (OBS_ONLY) block_store(gobs, obs_rows, nrow * D, tid, NT, wt);
    const bool norm = !OBS_ONLY && (pr.flags & MARLNAV_WRITE_OBS_NORM);
    // kBlockEarlyOut: a block with no finished env streams its rows and
    // states from waves 1..A-1 under wave 0's per-env phase (they have
    // nothing else to do there; blocks with finished envs keep the stores
    // after their re-init). early: this block's stores left early.
    bool early = false;
    if (!OBS_ONLY) {
        int *list = reinterpret_cast<int *>(lds + BP::LIST);
        int *flg = reinterpret_cast<int *>(lds + BP::FLG);
        const BlockEnvs<A, O, D> ev{st, lds + BP::OB, lds + BP::TG, obs_rows, e0};
        // ---- per-env reductions, terminal logic (wave 0, one lane per env)
        if (w == 0) {
            if (MARLNAV_ENV_PRIO) __builtin_amdgcn_s_setprio(MARLNAV_ENV_PRIO);  // (A/B builds)
            const bool env_on = l < ne;
            bool fin = false, tr_l = false, co_l = false, ta_l = false;
            if (env_on) {
                const int64_t e = e0 + l;
                float rx[A], ry[A];
                unsigned rf[A];
#pragma unroll
                for (int i = 0; i < A; ++i) {
                    const float4 t = red[A * l + i];
                    rx[i] = t.x;
                    ry[i] = t.y;
                    rf[i] = __float_as_uint(t.z);
                }
                const EnvEnd ee = env_end<A>([&](int i) { return rf[i]; }, lds[BP::SN + l],
                                             reinterpret_cast<const uint8_t *>(lds + BP::TM)[l],
                                             pr.trunc_after);
                const unsigned any_col = ee.any_col, all_in = ee.all_in;
                float rv[A];
#pragma unroll
                for (int i = 0; i < A; ++i) rv[i] = all_in ? ry[i] : rx[i];
                STAMPX(0);  // (wave 0: the reward terms read)
                const float rsum = torch_row_sum_r<A>(rv, [](float x) { return x; });
                const float rmean = rsum / (float)A;               // torch.mean (:233)

                const float step_num = ee.step_num;
                const bool truncated = ee.truncated, term_old = ee.term_old;
                const bool terminated = ee.terminated;
                fin = ee.fin;
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
                        float *obl = lds + BP::OB + 2 * O * l;
                        float *tgl = lds + BP::TG + 2 * l;
                        native_fresh_env<NOISY>(A, O, p, lds + BP::FORM,
                                                (uint64_t)(kl->a.env_offset + e), kl->a.step_idx,
                                                st + 5 * A * l, obl, tgl);
                        float *gob = kl->a.b.obstacles;
                        for (int i = 0; i < 2 * O; ++i) out_el(gob, e * O * 2 + i, obl[i]);
                        out_el(kl->a.b.target, 2 * e, tgl[0]);
                        out_el(kl->a.b.target, 2 * e + 1, tgl[1]);
                    }
                }
                const float sn_out = fin ? blend_in(step_num, 0.0f) : step_num;
                const uint8_t tm_out = (uint8_t)(!term_old && all_in);  // :218-219
                if (MARLNAV_AB & 1024) {  // (AB 1024: timing only, no per-env stores)
                } else if (MARLNAV_ENV_OUT && wt && full) {
                    // written through, 32-bit buffer offsets from the block's
                    // first env: no dirty L2 lines left for the end-of-launch
                    // write-back, and no 64-bit address math per store
                    // (MARLNAV_ENV_OUT, marlnav_debug.h)
                    wt_st(out_buf(bo.reward + e0, 4 * E), 4u * l, rmean);
                    wt_st(out_buf(bo.terminates + e0, E), (uint32_t)l, tm_out);
                    wt_st(out_buf(bo.terminated + e0, E), (uint32_t)l, (uint8_t)terminated);
                    wt_st(out_buf(bo.truncated + e0, E), (uint32_t)l, (uint8_t)truncated);
                    wt_st(out_buf(bo.step_num + e0, 4 * E), 4u * l, sn_out);
                } else {
                    out_el(bo.reward, e, rmean);
                    out_el(bo.terminates, e, tm_out);
                    out_el(bo.terminated, e, (uint8_t)terminated);
                    out_el(bo.truncated, e, (uint8_t)truncated);
                    out_el(bo.step_num, e, sn_out);
                }
                tr_l = truncated;
                co_l = any_col;
                ta_l = all_in;
            }
            STAMPX(1);  // (wave 0: the per-env outputs issued)
            const uint64_t finmask = __ballot(fin);
            early = kBlockEarlyOut<A, O, HELP> && overlap && full && !norm && finmask == 0ull;
            if (fin)
                list[__builtin_amdgcn_mbcnt_hi((unsigned)(finmask >> 32),
                                               __builtin_amdgcn_mbcnt_lo((unsigned)finmask, 0u))] = l;
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
            if (MARLNAV_ENV_PRIO) __builtin_amdgcn_s_setprio(0);
        } else if (overlap && !hw) {
            // ---- waves 1..A-1, while wave 0 runs the per-env phase: the
            // finished set from the inputs wave 0 uses (red flags, step_num,
            // terminates), then the native re-init (:104) and re-observation
            // (:105) of those envs. Disjoint LDS: wave 0 reads red/SN/TM; this
            // writes the states, obstacles, target and rows of finished envs.
            bool fin = false;
            if (l < ne) {  // (the same env_end as wave 0's, on the same LDS inputs)
                fin = env_end<A>([&](int i) { return __float_as_uint(red[A * l + i].z); },
                                 lds[BP::SN + l],
                                 reinterpret_cast<const uint8_t *>(lds + BP::TM)[l], pr.trunc_after)
                          .fin;
            }
            const uint64_t fm = __ballot(fin);
            early = kBlockEarlyOut<A, O, HELP> && full && !norm && fm == 0ull;
            if (early && !(MARLNAV_AB & 2))
                block_store2<E * A * D, E * A * 5, NT - 64>(
                    gobs, obs_rows, in_sgpr(bo.states_out + e0 * (A * 5)), st, tid - 64, wt);
            STAMPX(0);
            if (fm && !(MARLNAV_AB & 1)) {
                if (MARLNAV_REINIT_PRIO) __builtin_amdgcn_s_setprio(MARLNAV_REINIT_PRIO);  // (A/B builds)
                STAMPX(1);
                // kTailOut: the pass's obstacle / target outputs through the
                // block's SGPR pointers, written through (no dirty L2 lines
                // for the end-of-launch write-back)
                constexpr int kTailOut = MARLNAV_TAIL_PTRS >= 0 ? MARLNAV_TAIL_PTRS : (kPre ? 2 : 0);
                const TailOut tout{bo.obstacles, bo.target, e0, kTailOut == 2 && wt && full};
                reinit_reobs_native<A, O, kPre ? E : 0>(kargs_late<kHotKargsOff>(), ev,
                                                        lds + BP::FORM, MaskList{fm},
                                                        (int)__popcll(fm), pr.cap_distance,
                                                        tid - 64, NT - 64, lds + BP::FRESH,
                                                        kTailOut ? &tout : nullptr);
                STAMPX(2);
                if (MARLNAV_REINIT_PRIO) __builtin_amdgcn_s_setprio(0);
            }
        }
        __syncthreads();
        STAMP(4);
        const int nfin = flg[0];
        if (nfin && !overlap) {
            // ---- reference-RNG / noisy re-init (:104; noisy: done above by
            // wave 0) and observations of the re-initialised envs (:105)
            if (!NOISY) {
                if (!hw) reinit_block<A, O>(kargs_late<kHotKargsOff>(), ev, lds + BP::FORM, list, nfin, tid, NT);
                __syncthreads();
            }
            if (!hw) reobs_block<A, O>(ev, list, nfin, pr.cap_distance, tid, NT);
            __syncthreads();
        }
    }
    STAMP(5);
    // the one barrier after the per-env phase: the fused normaliser of a
    // block whose rows do not divide over its threads (partial block, or NT
    // not a multiple of D) stages mean and scale in LDS; every wave of the
    // block, the draw wave included, decides from this one value
    const bool norm_barrier = !OBS_ONLY && norm && !(full && NT % D == 0);
    if (hw) {  // (the draw wave stores nothing; it meets the norm path's barrier)
        if (norm_barrier) __syncthreads();
    } else if (!OBS_ONLY && full && !norm) {  // ---- stream the block out
        if (!(MARLNAV_AB & 2) && !early)
        block_store2<E * A * D, E * A * 5, NT>(gobs, obs_rows, in_sgpr(bo.states_out + e0 * (A * 5)),
                                               st, tid, wt);  // (E = 64: whole 16-byte pieces)
    } else if (!OBS_ONLY && full && NT % D == 0) {
        // ---- the same with the fused ObsNormalizer (utils.py:519-532):
        // thread tid only ever meets feature tid % D (NT is a multiple of D),
        // so its mean and scale are loaded once; every LDS read and every
        // division is issued ahead of the stores
        block_store2<E * A * D, E * A * 5, NT>(gobs, obs_rows, in_sgpr(bo.states_out + e0 * (A * 5)),
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
        if (norm_barrier) {  // (here: norm)
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
        block_store(in_sgpr(bo.states_out + e0 * (A * 5)), st, nrow * 5, tid, NT, wt);
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
    };  // block
    block();
}
