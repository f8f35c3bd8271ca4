/*
 * marlnav.h - C ABI of the MI355X (gfx950) environment-step library
 * (libmarlnav.so, built from marl-nav_amd/csrc/marlnav_step.hip).
 *
 * The reference (JussiM01/MARL-nav) has no FFI: its boundary is the Python
 * class `Env` (marlnav/environment.py:8-286). Each entry point below replaces
 * one method of that class; the file:line it replaces is given per function.
 * The Python host mirror (marl-nav_amd/environment.py) binds these with
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Every pointer in MarlnavStepBuffers and every array argument is a DEVICE
 *    pointer (hipMalloc / torch caching allocator), contiguous, fp32 / uint8
 *    as documented. The library never allocates, frees or synchronises.
 *  - Every call enqueues its work on `stream` (a hipStream_t; NULL = the
 *    default stream) and returns immediately.
 *  - Return value: 0 on success, a negative MARLNAV_E* code otherwise; the
 *    message is available from marlnav_last_error() (thread-local).
 *  - Shapes: P = num_parallel, A = num_agents, O = observed obstacles,
 *    S = obstacle_stride (obstacles stored per env, >= O),
 *    D = 2 + 2*O + 2*(A-1) observation features per agent.
 *  - The observation buffer is packed (P, A, D) in the field order of the
 *    reference's `Observations` namedtuple (utils.py:13-15), which is also the
 *    concatenation order of `ObsNormalizer` (utils.py:531):
 *      [target_angle | target_distance | obstacles_angles[O] |
 *       obstacles_distances[O] | others_angles[A-1] | others_distances[A-1]]
 */
#ifndef MARLNAV_H
#define MARLNAV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MARLNAV_ABI_VERSION 4

/* error codes */
#define MARLNAV_OK 0
#define MARLNAV_EINVAL (-1)  /* bad dims / params / null pointer */
#define MARLNAV_ELAUNCH (-2) /* HIP launch error */
#define MARLNAV_EUNSUPPORTED (-3)

/* MarlnavParams.flags */
/* Finished envs take their fresh agent states from the post-move states of
 * this step instead of fresh_states: reproduces the aliasing of
 * MockInitializer (utils.py:310-319) on the reference's first step, where
 * Env.states IS the initializer's tensor and _move_agents mutates it. */
#define MARLNAV_FRESH_STATES_FROM_MOVED 0x1u
/* Native re-init draws agent noise (TriangleIntitializer with
 * noisy_ags=True, utils.py:381-388). The reference ships noisy_ags=False
 * (utils.py:25). */
#define MARLNAV_NOISY_AGENTS 0x2u
/* Also write the ObsNormalizer output (utils.py:519-532) to obs_norm. */
#define MARLNAV_WRITE_OBS_NORM 0x4u
/* Apply ActionScaler (utils.py:535-547) to the actions on load: the kernel
 * reads policy actions in [-1, 1] and scales them itself. */
#define MARLNAV_SCALE_ACTIONS 0x8u

typedef struct MarlnavDims {
    int64_t num_parallel;    /* P  (environment.py:15)                        */
    int32_t num_agents;      /* A  (environment.py:16), 2 <= A <= 64          */
    int32_t num_obstacles;   /* O  observed per agent (environment.py:17,148) */
    int32_t obstacle_stride; /* S  = obstacles.shape[1], O <= S <= 256        */
    int32_t reserved;        /* must be 0                                     */
    int64_t env_offset;      /* global id of env 0 of this shard (native RNG) */
} MarlnavDims;

typedef struct MarlnavParams {
    /* dynamics bounds, environment.py:32-35 */
    float min_speed, max_speed, min_accel, max_accel;
    /* truncation: truncated = step_num > trunc_after, with
     * trunc_after = episode_len - 1 (environment.py:97) */
    float trunc_after;
    /* reward weights, environment.py:48-53 */
    float risk_factor, distance_factor, heading_factor;
    float target_factor, soft_factor, bond_factor;
    /* geometric constants, environment.py:56-68 */
    float ob_risk_dist, ag_risk_dist, ob_coll_dist, ag_coll_dist;
    float agents_min_d, agents_max_d, max_at_prop_d, max_angle_diff;
    float target_radius, cap_distance, bond_sharpness, ideal_dist, init_dist;
    /* native re-init of obstacles, utils.py:344-347, 390-398:
     * x = obs_range_x * (u - 0.5) + obs_mean_x (same for y) */
    float obs_range_x, obs_mean_x, obs_range_y, obs_mean_y;
    /* native noisy agents (MARLNAV_NOISY_AGENTS), utils.py:370-388:
     * pos += ags_dist * noise_std * N(0,1); heading rotated by
     * angle_range * (u - 0.5) */
    float ags_dist, noise_std, angle_range;
    /* ActionScaler (MARLNAV_SCALE_ACTIONS): a' = scale[k]*a + mean[k] */
    float act_scale[2], act_mean[2];
    uint32_t flags;
    uint32_t reserved;
    uint64_t seed;           /* native RNG seed: all 64 bits enter the Philox2x32-10
                                keys through splitmix64 + fmix32 */
} MarlnavParams;

typedef struct MarlnavStepBuffers {
    /* environment state, updated in place (environment.py:28-30, 38-39) */
    float *states;           /* (P, A, 5): x, y, dir_x, dir_y, speed       */
    float *obstacles;        /* (P, S, 2)                                  */
    float *target;           /* (P, 1, 2)                                  */
    float *step_num;         /* (P,)                                       */
    uint8_t *terminates;     /* (P,) bool: reach-target delayed flag       */
    /* inputs */
    const float *actions;    /* (P, A, 2): angle, acceleration             */
    /* reference-RNG re-init candidates (the init sampler's output of this
     * step, environment.py:78). NULL => native Philox re-init. Only the rows
     * of finished envs are read. */
    const float *fresh_states;    /* (P, A, 5) */
    const float *fresh_obstacles; /* (P, S, 2) */
    const float *fresh_target;    /* (P, 1, 2) */
    /* native re-init template: A*5 agent states then 2 target coords */
    const float *formation;
    /* outputs */
    float *obs;              /* (P, A, D) packed Observations              */
    float *reward;           /* (P,)                                       */
    uint8_t *terminated;     /* (P,) bool                                  */
    uint8_t *truncated;      /* (P,) bool                                  */
    /* episode statistics accumulators: 3 rows (trunc, col, tar) of
     * marlnav_counter_slots() uint64 partial sums, added to in place */
    uint64_t *counters;
    /* optional fused ObsNormalizer (MARLNAV_WRITE_OBS_NORM) */
    float *obs_norm;         /* (P, A, D)                                  */
    const float *norm_mean;  /* (D,)                                       */
    const float *norm_scale; /* (D,)                                       */
    /* optional observation template of a native fresh env (NULL: computed
     * in full): marlnav_formation_obs() of `formation`. Finished envs whose
     * agent rows and target re-initialise to the formation exactly (every
     * old value finite) take their target and agent-agent pairs from it and
     * compute only the agent-obstacle pairs. */
    const float *formation_obs; /* (A, A, 2)                               */
    /* optional second state buffer (NULL: `states` is updated in place): the
     * step reads `states` and writes every env's new state row here, so the
     * launch never writes the lines it read (a host double-buffers the two,
     * as the reference rebinds `states` each step, environment.py:80).
     * Must not overlap `states`. The env-block and pair-split kernels write
     * it with 16-byte vector stores and are chosen only when it is 16-byte
     * aligned (as `states` must be for them); otherwise the step falls back
     * to the generic wave kernel. */
    float *states_out;       /* (P, A, 5)                                  */
} MarlnavStepBuffers;

/* Env.step(actions) - environment.py:92-107 (with _move_agents :113-137,
 * observations :139-180, _rews_and_terms :184-269, _reinit :76-90).
 * step_idx keys the native RNG (any value when fresh_* are given). */
int marlnav_step(const MarlnavDims *dims, const MarlnavParams *params,
                 const MarlnavStepBuffers *bufs, uint64_t step_idx,
                 void *stream);

/* Env.observations() - environment.py:139-180. obs: (P, A, D). params:
 * the env's parameters (only cap_distance, environment.py:65 / :172-177,
 * is read); NULL means the reference's default cap 0.1. */
int marlnav_observe(const MarlnavDims *dims, const MarlnavParams *params,
                    const float *states, const float *obstacles,
                    const float *target, float *obs, void *stream);

/* Native TriangleIntitializer.__call__ for every env (utils.py:375-398), as
 * used by Env.__init__ (environment.py:26-30): writes states/obstacles/target
 * from the formation template and the Philox stream at step_idx. */
int marlnav_reinit_all(const MarlnavDims *dims, const MarlnavParams *params,
                       const float *formation, float *states,
                       float *obstacles, float *target, uint64_t step_idx,
                       void *stream);

/* Observation template of the native re-init's fresh env (the
 * TriangleIntitializer formation, utils.py:350-368, observed as in
 * environment.py:139-166): out[(a*A + m)*2 + {0, 1}] = (bearing before the
 * cap of environment.py:172-177, distance) of agent a to pair m, m = 0 the
 * target, m >= 1 the other agents in ascending order skipping a. The same
 * fp32 arithmetic as the step kernels' observation. formation: 5A + 2
 * floats (as MarlnavStepBuffers.formation); out: 2*A*A floats. */
int marlnav_formation_obs(const MarlnavDims *dims, const float *formation, float *out,
                          void *stream);

/* Number of uint64 partial-sum slots per counter row for these dims. */
int64_t marlnav_counter_slots(const MarlnavDims *dims);

/* Sum the counter slots: out3[0..2] = (num_trunc, num_col, num_tar)
 * (environment.py:43-45, 98, 210-211). out3 is a device pointer. */
int marlnav_counters_total(const MarlnavDims *dims, const uint64_t *counters,
                           uint64_t *out3, void *stream);

/* MAPPO._process_rewards (models.py:131-148) on the device. Discounted
 * returns of a rollout of T steps, G_t = done_t ? 0 : r_t + gamma * G_{t+1}
 * (G_T = 0), in float64 like the reference (its accumulator is
 * torch.zeros(P, dtype=float), models.py:133), then normalized in place,
 * returns = (G - mean) / (std + 1e-12) with the unbiased std over all T*P
 * values (torch.std_mean, models.py:140-144).
 *   rewards (T, P) fp32, done (T, P) uint8 (bool), returns (T, P) fp64 out,
 *   stats: 2 fp64 out (mean, std), work: marlnav_returns_work_size(P) fp64.
 * All device pointers; enqueued on stream. */
int64_t marlnav_returns_work_size(int64_t num_parallel);
int marlnav_discounted_returns(const float *rewards, const uint8_t *done, int64_t T,
                               int64_t P, double gamma, double *returns, double *stats,
                               double *work, void *stream);

/* Testing hook (not part of the reference's interface): restrict the step /
 * observe kernel selection to one family, process-wide. 0 = automatic (the
 * default); a family that does not support the call's shape or buffer
 * alignment falls back to the generic wave kernel. Returns the previous
 * setting. */
#define MARLNAV_FAMILY_AUTO 0
#define MARLNAV_FAMILY_BLOCK 1 /* env-block kernel (compiled shapes)          */
#define MARLNAV_FAMILY_SPLIT 2 /* pair-split kernel (compiled shapes)         */
/* 3 was the wave-tile family of ABI 1 (retired in ABI 2) */
#define MARLNAV_FAMILY_WAVE 4  /* generic wave kernel (any shape)             */
int marlnav_debug_force_family(int family);

/* Family (MARLNAV_FAMILY_*) the last marlnav_step / marlnav_observe call on
 * this thread launched. */
int marlnav_debug_last_family(void);

/* Testing hook (not part of the reference's interface): the step kernels'
 * bearing acos (environment.py:286) of the n consecutive fp32 bit patterns
 * from `first`, into the device array out[n] (tests/golden/acos_dev_check.py
 * compares it with the oracle's restatement over every fp32 in [-1, 1]). */
int marlnav_debug_acos_range(uint32_t first, int64_t n, float *out, void *stream);

/* Testing hook (not part of the reference's interface): the step kernels'
 * short fp32 division sequences (one Newton step, one residual correction:
 * the normalisation's two quotients, the reward terms' divisions by a
 * parameter, the bond term's reciprocal) against IEEE division, for the nd
 * divisor significands d_first + k * d_stride in [1, 2) and every dividend
 * significand; adds the mismatch counts to the device array out[3]
 * (quotients, parameter divisions, reciprocals). All-zero over the 2^23
 * divisors is the exhaustive proof (scripts/probes/div_exhaustive.hip). */
int marlnav_debug_fastdiv_check(uint32_t d_first, uint32_t d_stride, uint32_t nd, uint64_t *out,
                                void *stream);

/* Message of the last failing call on this thread. */
const char *marlnav_last_error(void);

/* MARLNAV_ABI_VERSION of the built library. */
int marlnav_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MARLNAV_H */
