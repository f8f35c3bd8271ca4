// kernel_lane.h - env-lane kernel prototype (A/B builds: MARLNAV_LANE_PROTO).
// Part of libmarlnav.so: included once, by marlnav_step.hip (one translation
// unit), inside its anonymous namespace.
#pragma once

// Lane = env: one wave steps 64 whole envs with no workgroup barrier - every
// agent's move, all A rows (A * (1 + O + A - 1) pairs per lane, two per
// pair2_fast) and the per-env phase in the lane's registers; the wave's
// inputs staged by LDS-DMA into its own LDS region, its rows and states
// transposed through LDS for 16-byte stores. Timing prototype: native re-init
// of finished envs is not done (their outputs are the un-re-initialised
// step's), the coordinate-checked pair math only.
template <int A, int O>
struct LanePlan {
    static constexpr int E = 64, D = 2 + 2 * O + 2 * (A - 1);
    static constexpr int ST = 0;                      // (E, A, 5)
    static constexpr int AC = ST + E * A * 5;         // (E, A, 2)
    static constexpr int OB = AC + E * A * 2;         // (E, O, 2)
    static constexpr int TG = OB + E * O * 2;         // (E, 2)
    static constexpr int SN = TG + E * 2;             // (E,)
    static constexpr int TM = SN + E;                 // (E,) bytes
    static constexpr int ROWS = (TM + E / 4 + 3) & ~3;  // (E, A, D) out
    static constexpr int STO = ROWS + E * A * D;      // (E, A, 5) out
    static constexpr int FLOATS = STO + E * A * 5;    // per wave
};

template <int A, int O>
__global__ void __launch_bounds__(256)
    lane_kernel(float *h_states, const float *h_actions, const float *h_obstacles,
                const float *h_target, const float *h_step_num, const uint8_t *h_terminates,
                int64_t h_P, KArgs k)
{
    using LP = LanePlan<A, O>;
    constexpr int E = LP::E, D = LP::D;
    (void)k;
    extern __shared__ __attribute__((aligned(16))) float lds_l[];
    const unsigned lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t tile = (int64_t)blockIdx.x * 4 + wv;
    const int64_t e0 = tile * E;
    if (e0 >= h_P) return;  // (the prototype's grids are whole waves: P % 64 == 0)
    float *L = lds_l + wv * LP::FLOATS;
    glds_span<E * A * 20>(h_states + e0 * (A * 5), L + LP::ST, lane);
    glds_span<E * A * 8>(h_actions + e0 * (A * 2), L + LP::AC, lane);
    glds_span<E * O * 8>(h_obstacles + e0 * (O * 2), L + LP::OB, lane);
    glds_span<E * 8>(h_target + e0 * 2, L + LP::TG, lane);
    glds_span<E * 4>(h_step_num + e0, L + LP::SN, lane);
    glds_span<E>(h_terminates + e0, L + LP::TM, lane);
    KArgsK *K = kargs_late<kHotKargsOff>();
    const MarlnavParams pr = load_params(K);
    const bool wt = (pr.flags & kWriteThroughFlag) != 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int l = (int)lane;
    float s[A * 5], ac[A * 2], ob[O * 2], tg[2];
#pragma unroll
    for (int i = 0; i < A * 5; ++i) s[i] = L[LP::ST + l * A * 5 + i];
#pragma unroll
    for (int i = 0; i < A * 2; ++i) ac[i] = L[LP::AC + l * A * 2 + i];
#pragma unroll
    for (int i = 0; i < O * 2; ++i) ob[i] = L[LP::OB + l * O * 2 + i];
    tg[0] = L[LP::TG + 2 * l];
    tg[1] = L[LP::TG + 2 * l + 1];
    const float sn_old = L[LP::SN + l];
    const uint8_t tm_old = reinterpret_cast<const uint8_t *>(L + LP::TM)[l];
    // ---- _move_agents (environment.py:113-123), every agent of the lane's env
    CoordRange crange;
#pragma unroll
    for (int i = 0; i < O * 2; ++i) crange.add(ob[i]);
    crange.add(tg[0]);
    crange.add(tg[1]);
#pragma unroll
    for (int a = 0; a < A; ++a) {
        float sn, c;
        sincos_k(clamp_t(ac[2 * a], -kPiF, kPiF), &sn, &c);
        const float dx = s[5 * a + 2], dy = s[5 * a + 3];
        const float ndx = c * dx + (-sn) * dy;
        const float ndy = sn * dx + c * dy;
        const float v = clamp_t(s[5 * a + 4] + clamp_t(ac[2 * a + 1], pr.min_accel, pr.max_accel),
                                pr.min_speed, pr.max_speed);
        s[5 * a] = s[5 * a] + ndx * v;
        s[5 * a + 1] = s[5 * a + 1] + ndy * v;
        s[5 * a + 2] = ndx;
        s[5 * a + 3] = ndy;
        s[5 * a + 4] = v;
        crange.add(s[5 * a]);
        crange.add(s[5 * a + 1]);
    }
    const bool fast = __ballot(!crange.ok()) == 0ull;
    // ---- observations + reward terms (:99-100)
    float rows[A][D];
    RowOut ro[A];
    bool unused = true;
    const bool refc = pr.bond_sharpness == 1.0f && pr.max_at_prop_d == 2.0f;
    (void)fast;
    (void)refc;
    // (timing prototype: the reference constants' coordinate-checked path only)
#pragma unroll
    for (int a = 0; a < A; ++a)
        ro[a] = observe_row_own<A, O, true, true, true>(s, ob, tg, a, s[5 * a], s[5 * a + 1],
                                                        s[5 * a + 2], s[5 * a + 3], rows[a], pr,
                                                        unused);
    // ---- per-env phase (:96-104, 213-233)
    float rx[A], ry[A];
    unsigned rf[A];
#pragma unroll
    for (int i = 0; i < A; ++i) {
        rx[i] = ro[i].r_miss;
        ry[i] = ro[i].r_hit;
        rf[i] = ro[i].flags;
    }
    const EnvEnd ee = env_end<A>([&](int i) { return rf[i]; }, sn_old, tm_old, pr.trunc_after);
    float rv[A];
#pragma unroll
    for (int i = 0; i < A; ++i) rv[i] = ee.all_in ? ry[i] : rx[i];
    const float rsum = torch_row_sum_r<A>(rv, [](float x) { return x; });
    const float rmean = rsum / (float)A;
    const float sn_out = ee.fin ? blend_in(ee.step_num, 0.0f) : ee.step_num;
    const uint8_t tm_out = (uint8_t)(!ee.term_old && ee.all_in);
    StepPtrs bo = load_ptrs(kargs_late<kHotKargsOff>());
    if (wt) {
        wt_st(out_buf(bo.reward + e0, 4 * E), 4u * l, rmean);
        wt_st(out_buf(bo.terminates + e0, E), (uint32_t)l, tm_out);
        wt_st(out_buf(bo.terminated + e0, E), (uint32_t)l, (uint8_t)ee.terminated);
        wt_st(out_buf(bo.truncated + e0, E), (uint32_t)l, (uint8_t)ee.truncated);
        wt_st(out_buf(bo.step_num + e0, 4 * E), 4u * l, sn_out);
    } else {
        out_el(bo.reward, e0 + l, rmean);
        out_el(bo.terminates, e0 + l, tm_out);
        out_el(bo.terminated, e0 + l, (uint8_t)ee.terminated);
        out_el(bo.truncated, e0 + l, (uint8_t)ee.truncated);
        out_el(bo.step_num, e0 + l, sn_out);
    }
    const unsigned c_trunc = __popcll(__ballot(ee.truncated));
    const unsigned c_col = __popcll(__ballot(ee.any_col != 0u));
    const unsigned c_tar = __popcll(__ballot(ee.all_in != 0u));
    if (lane == 0 && (c_trunc | c_col | c_tar)) {
        KArgsK *kl = kargs_late<kHotKargsOff>();
        uint64_t *cnt = kl->a.b.counters;
        const int64_t slots = kl->a.waves;
        if (cnt) {
            const int64_t sl = tile < slots ? tile : tile % slots;
            if (c_trunc) atomicAdd((unsigned long long *)&cnt[0 * slots + sl], (unsigned long long)c_trunc);
            if (c_col) atomicAdd((unsigned long long *)&cnt[1 * slots + sl], (unsigned long long)c_col);
            if (c_tar) atomicAdd((unsigned long long *)&cnt[2 * slots + sl], (unsigned long long)c_tar);
        }
    }
    // ---- rows and states through LDS, then 16-byte stores
#pragma unroll
    for (int a = 0; a < A; ++a) lds_row_write<D>(L + LP::ROWS + (l * A + a) * D, rows[a]);
#pragma unroll
    for (int i = 0; i < A * 5; ++i) L[LP::STO + l * A * 5 + i] = s[i];
    wave_sync();
    constexpr int Q1 = E * A * D / 4, Q2 = E * A * 5 / 4;
    const float4 *r4 = reinterpret_cast<const float4 *>(L + LP::ROWS);
    const float4 *s4 = reinterpret_cast<const float4 *>(L + LP::STO);
    float4 v1[(Q1 + 63) / 64], v2[(Q2 + 63) / 64];
#pragma unroll
    for (int kq = 0; kq < (Q1 + 63) / 64; ++kq)
        if ((kq + 1) * 64 <= Q1 || l + kq * 64 < Q1) v1[kq] = r4[l + kq * 64];
#pragma unroll
    for (int kq = 0; kq < (Q2 + 63) / 64; ++kq)
        if ((kq + 1) * 64 <= Q2 || l + kq * 64 < Q2) v2[kq] = s4[l + kq * 64];
    const OutBuf o1 = out_buf(bo.obs + e0 * (A * D), Q1 * 16), o2 = out_buf(bo.states_out + e0 * (A * 5), Q2 * 16);
#pragma unroll
    for (int kq = 0; kq < (Q1 + 63) / 64; ++kq)
        if ((kq + 1) * 64 <= Q1 || l + kq * 64 < Q1) wt_st4(o1, 16u * (l + kq * 64), v1[kq]);
#pragma unroll
    for (int kq = 0; kq < (Q2 + 63) / 64; ++kq)
        if ((kq + 1) * 64 <= Q2 || l + kq * 64 < Q2) wt_st4(o2, 16u * (l + kq * 64), v2[kq]);
}
