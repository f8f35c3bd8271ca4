// kernel_wave.h - generic wave kernel (any shape, any alignment).
// Part of libmarlnav.so: included once, by marlnav_step.hip (one translation
// unit), inside its anonymous namespace.
#pragma once

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
    const bool wt = (pr.flags & kWriteThroughFlag) != 0;  // written-through outputs
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
        if (row_on) {
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
                out_el(b.reward, e, rsum / (float)A);                     // torch.mean (:233)

                float step_num = step_num_in + 1.0f;               // :96
                const bool truncated = step_num > pr.trunc_after;  // :97
                const bool term_old = term_in != 0;
                const bool terminated = any_col || term_old;       // :213-214
                out_el(b.terminates, e, (uint8_t)(!term_old && all_in));  // :218-219
                out_el(b.terminated, e, (uint8_t)terminated);
                out_el(b.truncated, e, (uint8_t)truncated);
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
                out_el(b.step_num, e, step_num);
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
                store_row<D_T>(b.obs + (e0 * A + lane) * D_T, rowv, wt);
                if (norm) {
                    float nv[D_T];
#pragma unroll
                    for (int k = 0; k < D_T; ++k)
                        nv[k] = (rowv[k] - b.norm_mean[k]) / b.norm_scale[k];
                    store_row<D_T>(b.obs_norm + (e0 * A + lane) * D_T, nv, wt);
                }
            }
        } else if (wp.obs_lds)
            wave_store(b.obs + e0 * A * D, obs_t, nr * D, lane,
                       norm ? b.obs_norm + e0 * A * D : nullptr, b.norm_mean, b.norm_scale, D, wt);
        else if (norm && row_on)
            for (int k = 0; k < D; ++k)
                b.obs_norm[(e0 * A + lane) * D + k] =
                    (out_row[k] - b.norm_mean[k]) / b.norm_scale[k];
        if (!OBS_ONLY)
            wave_store((b.states_out ? b.states_out : b.states) + e0 * A * 5, st, nr * 5, lane,
                       nullptr, nullptr, nullptr, 1, wt);
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
        *STAMP_PTR((size_t)gw * 24 + 16) = t_entry;
        *STAMP_PTR((size_t)gw * 24 + 17) = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        *STAMP_PTR((size_t)gw * 24 + 18) = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
    }
#endif
}
