// marlnav_debug.h - diagnostic stamps build (MARLNAV_STAMPS=1, scripts/kstamps.py); compiles to nothing otherwise.
// Part of libmarlnav.so: included once, by marlnav_step.hip (one translation
// unit), inside its anonymous namespace.
#pragma once

// Diagnostic build (MARLNAV_STAMPS=1, scripts/kstamps.py): lane 0 of every
// wave records s_memrealtime / s_memtime at each phase boundary into a
// buffer registered with marlnav_debug_stamps().
#ifndef MARLNAV_STAMPS
#define MARLNAV_STAMPS 0
#endif
#if MARLNAV_STAMPS
__device__ unsigned long long *g_stamps;
// global (not flat) stores: a flat store also counts in lgkmcnt, so the next
// LDS wait would wait for the stamp's write to reach memory
typedef __attribute__((address_space(1))) unsigned long long stamp_t;
#define STAMP_PTR(off) ((stamp_t *)(g_stamps) + (off))
#define STAMP(k)                                                                   \
    do {                                                                           \
        if (lane == 0) {                                                           \
            stamp_t *sp_ = STAMP_PTR((size_t)gw * 24);                             \
            sp_[2 * (k)] = wall_clock64();                                         \
            sp_[2 * (k) + 1] = clock64();                                          \
        }                                                                          \
    } while (0)
// extra realtime-only stamps at slots 20..23 (diagnostic sub-phases): the
// per-env / re-init sub-phases (STAMPX), or with MARLNAV_SUBSTAMPS=1 the
// env-block kernel's stage and observe sub-phases (STAMPS_S) instead
#ifndef MARLNAV_SUBSTAMPS
#define MARLNAV_SUBSTAMPS 0
#endif
#define STAMP_SLOT_(k)                                                             \
    do {                                                                           \
        if (lane == 0) *STAMP_PTR((size_t)gw * 24 + 20 + (k)) = wall_clock64();    \
    } while (0)
#if MARLNAV_SUBSTAMPS
#define STAMPX(k) \
    do {          \
    } while (0)
#define STAMPS_S(k) STAMP_SLOT_(k)
#else
#define STAMPX(k) STAMP_SLOT_(k)
#define STAMPS_S(k) \
    do {            \
    } while (0)
#endif
#else
#define STAMPS_S(k) \
    do {            \
    } while (0)
#define STAMPX(k) \
    do {          \
    } while (0)
#define STAMP(k) \
    do {         \
    } while (0)
#endif

// Timing-only ablation switches of A/B variant builds (scripts/build_variant.sh
// ... -DMARLNAV_AB=bits); 0 in the product build.
#ifndef MARLNAV_AB
#define MARLNAV_AB 0
#endif
// A/B variant (not timing-only): every workgroup-spread shape of the split
// kernel finishes each row's reward on its row leader (kSplitRRLeader)
#ifndef MARLNAV_SPLIT_RR_LEADER
#define MARLNAV_SPLIT_RR_LEADER 0
#endif
#ifndef MARLNAV_AB_NOREFC
#define MARLNAV_AB_NOREFC 0
#endif
// Env-block kernel: wave 0's per-env phase (the block's latency chain while
// its other waves wait at the barrier) at this s_setprio over the other
// blocks' waves on its SIMD. A/B (profiles/r04_ab_env_prio.txt, graph
// replay, steady / fresh): 0 -> 3: 65536x3x3 7.00 -> 6.95 / 7.24 -> 7.16 us,
// 16384x3x3 5.34 -> 5.30 / 5.36 -> 5.34 us.
#ifndef MARLNAV_ENV_PRIO
#define MARLNAV_ENV_PRIO 3
#endif
// Env-block kernel: wave 0's per-env outputs (reward, terminates,
// terminated, truncated, step_num; environment.py:96-104, 213-233) of a full
// block in a written-through launch as written-through buffer stores (1) or
// as plain stores (0). Same box, graph replay, steady (profiles/r05_ab_envout.txt):
// 0 -> 1: 65536x3x3 6.84 -> 6.70 us, 16384x3x3 5.01 -> 4.99, 32768x3x3 and
// 131072x3x8 unchanged. Staging them in LDS and storing them as 16-byte
// written-through pieces beside the block store instead measured slower
// (6.94, 5.13, 17.89 us). The split kernel's per-env outputs written through
// the same way (removed) measured slower: 4096x16x32 11.63 -> 11.80 us,
// 512x16x32 8.00 -> 8.17, 1024x3x8 4.82 -> 4.90 (profiles/r05_ab_envout_confirm.txt).
#ifndef MARLNAV_ENV_OUT
#define MARLNAV_ENV_OUT 1
#endif
// Split kernel, one env per wave (A16/O32): observation in two passes, a
// finished env re-initialised and re-observed by its own wave before the
// per-env barrier (kSplitOwn, kernel_split.h)
#ifndef MARLNAV_SPLIT_OWN
#define MARLNAV_SPLIT_OWN 0  // 1: the default split instantiation too (A/B builds)
#endif
#ifndef MARLNAV_LATE_PTRS
#define MARLNAV_LATE_PTRS 1  // 0: block kernel output pointers held from the entry (A/B builds)
#endif
#ifndef MARLNAV_SPLIT_OWN_MAX
#define MARLNAV_SPLIT_OWN_MAX 2048  // the own-wave instantiation for A16/O32 grids of at most this many envs
#endif
#ifndef MARLNAV_SPLIT_FORM_LDS
#define MARLNAV_SPLIT_FORM_LDS 0  // 1: the split kernel's fused A3 re-init reads the formation from LDS (A/B)
#endif
#ifndef MARLNAV_DRAW_WAVE
#define MARLNAV_DRAW_WAVE 1  // 0: no draw-wave block instantiation (A/B builds)
#endif
#ifndef MARLNAV_TPL_LOADS_FIRST
#define MARLNAV_TPL_LOADS_FIRST 1  // 0: the template re-init pass interleaves its LDS reads and writes (r05 A/B)
#endif
#ifndef MARLNAV_OWN_VPIN
#define MARLNAV_OWN_VPIN 1  // own-wave split instantiation's parameters in VGPRs (0: off; 2: every split kernel, A/B)
#endif
#ifndef MARLNAV_SPLIT_EARLY
#define MARLNAV_SPLIT_EARLY 1  // 0: own-wave split tiles stored after the per-env phase (A/B builds;
                               // early: 8.38 vs 8.48 us at 2048x16x32, profiles/r05_ab_early.txt)
#endif
#ifndef MARLNAV_SPLIT_OWN_OFF
#define MARLNAV_SPLIT_OWN_OFF 0  // 1: never pick the kSplitOwn instantiation (A/B builds)
#endif
// Env-block kernel: the finished-env pass's obstacle / target stores through
// the block's SGPR pointers (1), also written through (2), or through kernarg
// loads as plain stores (0); -1: 2 where the fresh obstacles are drawn at
// stage time (O <= A), else 0. Same box, graph replay, steady
// (profiles/r05_ab_tp2rp.txt): 0 -> 2: 16384x3x3 5.01 -> 4.89 us, 32768x3x3
// 5.70 -> 5.55, 65536x3x3 6.70 -> 6.70, 131072x3x8 17.12 -> 17.89 (its
// 16 obstacle stores per finished env written through); 0 -> 1: 65536x3x3
// 6.72 -> 6.83 (profiles/r05_ab_tp_sprio_own.txt).
#ifndef MARLNAV_TAIL_PTRS
#define MARLNAV_TAIL_PTRS -1
#endif
// Split kernel: s_setprio of wave 0's row rewards and per-env phase (A/B builds)
#ifndef MARLNAV_SPLIT_PRIO
#define MARLNAV_SPLIT_PRIO 0
#endif
// Env-block kernel: s_setprio of the re-init waves' pass in blocks with
// finished envs (0: none; A/B builds)
#ifndef MARLNAV_REINIT_PRIO
#define MARLNAV_REINIT_PRIO 0
#endif
// Round-4 A/B variants measured and removed from the sources (in git history
// at bc24ae1, DESIGN.md §5 "Round 4"): MARLNAV_EARLY_OUT's first forms,
// MARLNAV_DEFER_BLOCK_ENV_OUT, MARLNAV_TAIL_PRIO (env-block kernel);
// MARLNAV_SPLIT_OVERLAP, MARLNAV_SPLIT_OWN_ENV, MARLNAV_SPLIT_DEFER_ENV_OUT,
// MARLNAV_SPLIT_ENV_PRIO (split kernel); MARLNAV_DEFER_REINIT_OUT (re-init).
// Round 6 (HISTORY.md; code in git history at 9a7feb1): MARLNAV_ONE_STAGE
// (each wave gathers its agent's rows by per-lane dword LDS-DMA and moves it
// before ONE barrier: bit-exact, slower at every shape, 65536x3x3 6.55 ->
// 6.89 us, 16384x3x3 4.65 -> 4.73, 2^20 envs 68.7 -> 74.4). Round 6, code in
// git history at a9bbeb6 (profiles/r06_ab_*.txt, r06_claim_probe.txt):
// MARLNAV_STAGGER (late blocks per CU: never faster), MARLNAV_PAIR_SPLIT (two
// waves per agent, the row's pairs split: bit-exact, 16384x3x3 4.65 ->
// 4.67-4.75 us), MARLNAV_STAGE_AUX (staging cache policy: +-0 or slower),
// MARLNAV_ACT_FIRST (action loads before the spans: +0.1 us),
// MARLNAV_CNT_EARLY (+-0), MARLNAV_BLOCK_TILES (T blocks per workgroup:
// bit-exact, 65536x3x3 6.48 -> 7.38 / 7.67 us), MARLNAV_CLAIM_PROBE (split
// kernel: the claim of a cross-workgroup work list, +0.35 us at 4096x16x32);
// at 7e0c2a8: MARLNAV_LANE_PROTO (kernel_lane.h, an env-lane kernel: one wave per
// 64 whole envs, no block barrier; slower at every size, 65536x3x3 6.51 ->
// 7.20 us without its re-init); at c5c92fc: MARLNAV_RMOVE (draw-wave
// instantiation: every lane moves all A agents of its env, no move barrier;
// bit-exact, +0.4 us at 16384x3x3); at 16437ed: MARLNAV_BLOCK_PIPE (two
// env blocks per workgroup, software-pipelined: bit-exact, 65536x3x3 6.44 ->
// 9.45 us, profiles/r06_ab_pipe.txt); at eb3feb8: MARLNAV_SPLIT_SPEC (split
// kernel A3/O8: a finished env's fresh rows from obstacle pairs computed
// speculatively for every env; bit-exact, 1024x3x8 4.85 -> 4.85-4.94 us,
// profiles/r06_ab_split_spec.txt).
// Round 5 (DESIGN.md §5 "Round 5"; code in git history at deae14b):
// MARLNAV_BLOCK_ENV_ROT / MARLNAV_SPLIT_ENV_ROT (the per-env phase on wave
// block % A / workgroup % 4: no gain, and the general re-init thread index
// alone changed the block kernel's register allocation, +0.17 us at
// 65536x3x3), MARLNAV_SPLIT_OWN_REINIT (A16/O32: a finished env re-initialised
// and re-observed by its own wave before the per-env barrier: bit-exact, but
// 4096x16x32 11.66 -> 14.51 us, the lone wave's pair chains run one after the
// other), MARLNAV_SPLIT_ENV_WT.
// Env-block kernel: blocks with no finished env stream their rows from waves
// 1..A-1 under the per-env phase (1), after it (0), or by shape (-1: the
// product's choice, kBlockEarlyOut in kernel_block.h)
#ifndef MARLNAV_EARLY_OUT
#define MARLNAV_EARLY_OUT -1
#endif
// Packed pair math (pair2_fast: two pairs of a row per v_pk_*_f32) in the
// coordinate-checked observation of the env-block kernel (1), or one pair per
// VALU instruction (0; A/B builds). scripts/probes/pair_forms.hip. Same box,
// graph replay, steady (profiles/r06_ab_packed.txt): 131072x3x8 16.61 ->
// 16.06 us, 65536x3x3 6.36 -> 6.35, 16384x3x3 4.62 -> 4.61.
#ifndef MARLNAV_PACKED_PAIRS
#define MARLNAV_PACKED_PAIRS 1
#endif
// The same in the pair-split kernel's split_pairs (A16/O32, A3/O8 small
// grids): 4096x16x32 11.19 -> 11.33 us, 1024x3x8 and 2048x16x32 unchanged
// (profiles/r06_ab_packed_split.txt): off (A/B builds: 1)
#ifndef MARLNAV_PACKED_SPLIT
#define MARLNAV_PACKED_SPLIT 0
#endif
