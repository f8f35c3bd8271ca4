// kernel_args.h - kernel-argument block of the compiled-shape kernels and LDS-DMA staging helpers.
// Part of libmarlnav.so: included once, by marlnav_step.hip (one translation
// unit), inside its anonymous namespace.
#pragma once

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

// Kernarg pointer the compiler cannot hoist loads through. OFF: byte offset
// of the KArgs argument in the kernarg segment (the env-block and pair-split
// kernels pass their staging pointers first, kHotKargsOff).
template <int OFF>
__device__ __forceinline__ KArgsK *kargs_late()
{
    const char *p = (const char *)__builtin_amdgcn_kernarg_segment_ptr() + OFF;
    KArgsK *k = (KArgsK *)p;
    asm volatile("" : "+s"(k));
    return k;
}

// The env-block and pair-split kernels' leading kernel arguments: the
// pointers their staging reads and the env count, 14 dwords that the
// dispatcher preloads into user SGPRs (Makefile:
// -amdgpu-kernarg-preload-count=14), so a wave's first LDS-DMA does not wait
// for a scalar load of the kernarg segment (65536x3x3 8.72 -> 8.47 us
// median, A/B on one box). KArgs follows at kHotKargsOff.
constexpr int kHotKargsOff = 7 * 8;

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
    float *states, *states_out, *obstacles, *target, *step_num, *obs, *reward;
    uint8_t *terminates, *terminated, *truncated;
    const float *actions, *formation;
};

__device__ __forceinline__ StepPtrs load_ptrs(KArgsK *K)
{
    StepPtrs q;
    q.states = K->a.b.states;
    q.states_out = K->a.b.states_out;  // = states unless double-buffered (marlnav_step)
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
template <int NB, int AUX = 0>
__device__ __forceinline__ void glds_span(const void *src, float *dst, unsigned lane)
{
    constexpr int N16 = NB / 16, R4 = (NB % 16) / 4;
#pragma unroll
    for (int k = 0; k * 64 < N16; ++k) {
        const char *s = in_sgpr(reinterpret_cast<const char *>(src) + k * 1024);
        if ((k + 1) * 64 <= N16 || (int)lane < N16 - k * 64)
            __builtin_amdgcn_global_load_lds(s + lane * 16u, (LdsVoid *)(dst + k * 256), 16, 0,
                                             AUX);
    }
    if constexpr (R4 > 0) {
        const char *s = in_sgpr(reinterpret_cast<const char *>(src) + N16 * 16);
        if ((int)lane < R4)
            __builtin_amdgcn_global_load_lds(s + lane * 4u, (LdsVoid *)(dst + N16 * 4), 4, 0,
                                             AUX);
    }
}

// s_waitcnt vmcnt(n) for a wave-uniform n (0..7; larger waits for all)
__device__ __forceinline__ void wait_vmcnt(int n)
{
    switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
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
