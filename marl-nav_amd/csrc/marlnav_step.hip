// marlnav_step.hip - gfx950 (MI355X) kernels behind include/marlnav.h: the
// library's one translation unit for the step.
//
// One launch performs the whole Env.step of the reference
// (marlnav/environment.py:92-107): heading/speed integration, every
// agent->target/obstacle/agent distance and bearing, the reward terms, the
// terminal logic, the masked re-initialisation of finished envs and the
// recomputed observations of those envs.
//
// Three kernel families, one launch per step, picked on the
// host by shape, grid size and buffer alignment (marlnav_step, end of file):
//   block_kernel  (kernel_block.h) - one workgroup of A waves per 64
//                   consecutive envs, lane = env, wave = agent: the compiled
//                   A3 shapes, the headline path;
//   split_kernel  (kernel_split.h) - LPR lanes per agent row, wave-private
//                   tiles: A16/O32, and A3 grids too small to fill the chip;
//   wave_kernel   (kernel_wave.h) - any runtime shape, any alignment.
// device_math.h holds the arithmetic they share, kernel_reinit.h the
// workgroup-spread re-init / re-observation, kernel_args.h the argument
// block and LDS-DMA staging, marlnav_debug.h the stamps diagnostic build.
// All stage their inputs in LDS, keep a lane's own row in registers,
// assemble the packed observation rows in LDS where they stream out with
// 16-byte stores, and re-initialise / re-observe only the envs that
// finished. No MFMA: nothing here contracts.
//
// Numerics: built with -ffp-contract=off and the HIP default
// correctly rounded fp32 division and sqrt, so every distance, dot product
// and reward term is the fp32 expression the reference's CPU path evaluates,
// summed in torch's order. sin/cos of the heading update are correctly
// rounded (fp64 evaluation rounded once, sincos_k, the same operation
// sequence as oracle_sincos in oracle/marlnav_oracle.c; the reference's MKL
// VML sin/cos agrees with it on 95% of angles); acos is the device libm's
// acosf.
#include <hip/hip_runtime.h>

#include <atomic>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/marlnav.h"

namespace {

constexpr float kPiF = 3.14159265358979323846f;
constexpr int kMaxAgents = 64;
constexpr int kMaxStride = 256;
constexpr int kWavesPerBlock = 4;
constexpr int kWaveLdsFloats = 4096;    // 16 KiB per wave, 64 KiB per block
constexpr int kObsTileMax = 2304;       // floats of packed obs staged per wave

#include "marlnav_debug.h"

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
}  // namespace

// error reporting shared with the other translation units of the library
__attribute__((visibility("hidden"))) int marlnav_internal_fail(int code, const char *msg)
{
    return fail(code, "%s", msg);
}

namespace {

#include "device_math.h"
#include "kernel_wave.h"
#include "kernel_args.h"
#include "kernel_reinit.h"
#include "kernel_split.h"
#include "kernel_block.h"

// ----------------------------------------------------- native reinit kernel
__global__ void reinit_all_kernel(int64_t P, int A, int S, int64_t env_offset, uint64_t sidx,
                                  MarlnavParams pr, const float *__restrict__ formation,
                                  float *states, float *obstacles, float *target)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P) return;
    if (pr.flags & MARLNAV_NOISY_AGENTS)
        native_fresh_env<true, false>(A, S, pr, formation, (uint64_t)(env_offset + e), sidx,
                               states + e * A * 5, obstacles + e * S * 2, target + 2 * e);
    else
        native_fresh_env<false, false>(A, S, pr, formation, (uint64_t)(env_offset + e), sidx,
                                states + e * A * 5, obstacles + e * S * 2, target + 2 * e);
}

// marlnav_formation_obs: one thread per (agent a, pair m) of the formation;
// the IEEE pair math, equal to every kernel's (the short sequences agree
// with it wherever they run); cap 0 leaves the bearing uncapped
__global__ void formation_obs_kernel(int A, const float *__restrict__ form, float *__restrict__ out)
{
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= A * A) return;
    const int a = i / A, m = i - a * A;
    const float ox = form[5 * a], oy = form[5 * a + 1];
    const float dx = form[5 * a + 2], dy = form[5 * a + 3];
    float px = form[5 * A], py = form[5 * A + 1];
    if (m > 0) {
        const int k = (m - 1) + (m - 1 >= a ? 1 : 0);
        px = form[5 * k];
        py = form[5 * k + 1];
    }
    bool unused = true;
    const float d = pair_dist<false>(ox, oy, px, py, unused);
    out[2 * i] = pair_angle<false>(ox, oy, px, py, dx, dy, d, 0.0f, unused);
    out[2 * i + 1] = d;
}

// marlnav_debug_acos_range: the bearing acos of consecutive fp32 patterns
__global__ void acos_range_kernel(uint32_t first, int64_t n, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = acos_k(__uint_as_float(first + (uint32_t)i));
}

// marlnav_debug_fastdiv_check: the step kernels' short division sequences
// (div2_fast, div_c with make_divc, recip_fast; device_math.h) against IEEE
// division, for the d significands d_first + k * d_stride (k < gridDim.x) in
// [1, 2) and EVERY x significand in [1, 2) - the pairs that decide every
// guarded case (the sequences are scale- and sign-invariant inside the
// guards). out[0..2] += mismatching (x, d) pairs of div2_fast, div_c, and
// mismatching d of recip_fast.
__global__ void __launch_bounds__(256) fastdiv_check_kernel(uint32_t d_first, uint32_t d_stride,
                                                            unsigned long long *__restrict__ out)
{
    const uint32_t dm = (d_first + blockIdx.x * d_stride) & 0x7FFFFFu;
    const float d = __uint_as_float(0x3f800000u | dm);
    bool ok = true;
    const DivC dc = make_divc(d, ok);
    unsigned long long b_div2 = 0, b_divc = 0;
    if (threadIdx.x == 0 &&
        __float_as_uint(recip_fast(d, ok)) != __float_as_uint(1.0f / d))
        atomicAdd(&out[2], 1ull);
    for (uint32_t xm = threadIdx.x; xm < (1u << 23); xm += 2 * blockDim.x) {
        const float x = __uint_as_float(0x3f800000u | xm);
        const float y = __uint_as_float(0x3f800000u | (xm + blockDim.x));
        float qx, qy;
        div2_fast(x, y, d, &qx, &qy, ok);
        b_div2 += (__float_as_uint(qx) != __float_as_uint(x / d)) +
                  (__float_as_uint(qy) != __float_as_uint(y / d));
        b_divc += __float_as_uint(div_c(x, dc, ok)) != __float_as_uint(x / d);
        b_divc += __float_as_uint(div_c(y, dc, ok)) != __float_as_uint(y / d);
    }
    for (int o = 32; o > 0; o >>= 1) {
        b_div2 += __shfl_xor(b_div2, o);
        b_divc += __shfl_xor(b_divc, o);
    }
    if ((threadIdx.x & 63) == 0) {
        if (b_div2) atomicAdd(&out[0], b_div2);
        if (b_divc) atomicAdd(&out[1], b_divc);
    }
    if (!ok && threadIdx.x == 0) atomicAdd(&out[2], 1ull << 32);  // (a guard refused: never here)
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
struct Launch {
    int W;
    int64_t ntiles, waves, blocks;
    WavePlan plan;
};

// envs per wave tile: 64 / A, rounded down to a multiple of 4 when that
// leaves >= 4 (16-byte aligned tiles), then shrunk to the LDS budget
bool has_variant(int A, int O);

bool rows_in_registers(int A, int O)
{
    return has_variant(A, O) && obs_dim(A, O) <= kRowRegsMaxD;
}

int pick_wave_envs(int A, int O, int S)
{
    int W = 64 / A;
    if (W >= 4) W &= ~3;
    const bool rr = rows_in_registers(A, O);
    while (W > 1 && make_plan(W, A, O, S, rr).floats > kWaveLdsFloats) W >>= 1;
    return W < 1 ? 1 : W;
}

Launch plan_launch(const MarlnavDims *d)
{
    Launch L;
    L.W = pick_wave_envs(d->num_agents, d->num_obstacles, d->obstacle_stride);
    L.plan = make_plan(L.W, d->num_agents, d->num_obstacles, d->obstacle_stride,
                       rows_in_registers(d->num_agents, d->num_obstacles));
    L.ntiles = (d->num_parallel + L.W - 1) / L.W;
    L.waves = (L.ntiles + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock;
    L.blocks = L.waves / kWavesPerBlock;
    return L;
}

int validate(const MarlnavDims *d)
{
    if (!d) return fail(MARLNAV_EINVAL, "dims is NULL");
    if (d->num_parallel < 1)
        return fail(MARLNAV_EINVAL, "num_parallel=%lld < 1", (long long)d->num_parallel);
    if (d->num_agents < 2 || d->num_agents > kMaxAgents)
        return fail(MARLNAV_EINVAL, "num_agents=%d outside [2, %d]", d->num_agents, kMaxAgents);
    if (d->num_obstacles < 1 || d->num_obstacles > d->obstacle_stride)
        return fail(MARLNAV_EINVAL, "num_obstacles=%d outside [1, obstacle_stride=%d]",
                    d->num_obstacles, d->obstacle_stride);
    if (d->obstacle_stride > kMaxStride)
        return fail(MARLNAV_EINVAL, "obstacle_stride=%d > %d", d->obstacle_stride, kMaxStride);
    const Launch L = plan_launch(d);
    if (L.plan.floats > kWaveLdsFloats)
        return fail(MARLNAV_EUNSUPPORTED, "wave tile does not fit LDS for A=%d O=%d S=%d",
                    d->num_agents, d->num_obstacles, d->obstacle_stride);
    return 0;
}

using StepFn = void (*)(StepArgs, MarlnavParams);

struct KernelPair {
    int A, O;
    StepFn step, obs, noisy;
};

const KernelPair kVariants[] = {
    {3, 3, wave_kernel<3, 3, false>, wave_kernel<3, 3, true>, wave_kernel<3, 3, false, true>},
    {3, 8, wave_kernel<3, 8, false>, wave_kernel<3, 8, true>, wave_kernel<3, 8, false, true>},
    {3, 1, wave_kernel<3, 1, false>, wave_kernel<3, 1, true>, wave_kernel<3, 1, false, true>},
    {2, 1, wave_kernel<2, 1, false>, wave_kernel<2, 1, true>, wave_kernel<2, 1, false, true>},
    {16, 32, wave_kernel<16, 32, false>, wave_kernel<16, 32, true>,
     wave_kernel<16, 32, false, true>},
};

// Step kernels that take their arguments through one KArgs block
// the env-block and pair-split kernels: staging pointers and P first
// (kHotKargsOff, kernel_args.h), then KArgs
using BlockFn = void (*)(float *, const float *, const float *, const float *, const float *,
                         const uint8_t *, int64_t, KArgs);
// the kernarg layout places each argument at its natural alignment: six
// pointers and an int64 (56 bytes), then KArgs - where kargs_late reads it
static_assert(6 * sizeof(float *) + sizeof(int64_t) == kHotKargsOff && alignof(KArgs) <= 8,
              "KArgs must follow the seven preloaded arguments at kHotKargsOff");

bool aligned(const void *p, uintptr_t n) { return (reinterpret_cast<uintptr_t>(p) & (n - 1)) == 0; }

// pair-split kernels (split_kernel): rows with many pairs, or grids too small
// for one lane per row to fill the chip
struct SplitVariant {
    int A, O, epw;
    BlockFn step, obs, noisy;
    size_t lds;
    bool always;  // also for large grids
    int lpr;
    BlockFn step_own;  // kSplitOwn instantiation (one env per wave), or null
};

#define MARLNAV_SPLIT_VARIANT(A, O, LPR, ALWAYS)                                          \
    {A, O, SplitPlan<A, O, LPR>::EPW, split_kernel<A, O, LPR, false, false>,             \
     split_kernel<A, O, LPR, true, false>, split_kernel<A, O, LPR, false, true>,         \
     (size_t)(SplitPlan<A, O, LPR>::FLOATS * kWavesPerBlock + SplitPlan<A, O, LPR>::BLK) * 4, \
     ALWAYS, LPR,                                                                        \
     kSplitOwnShape<A, O, LPR> ? split_kernel<A, O, LPR, false, false, true> : nullptr}
const SplitVariant kSplitVariants[] = {
    MARLNAV_SPLIT_VARIANT(16, 32, 4, true),
    MARLNAV_SPLIT_VARIANT(3, 8, 4, false),
    MARLNAV_SPLIT_VARIANT(3, 3, 4, false),
    // 8 lanes per row (<= 2 pairs per lane) for grids of at most kSplitTinyWaves
    // LPR=4 waves (measured: 2x3x3 3.89 -> 3.44 us, 1024x3x8 6.31 -> 6.14 us;
    // 2048x3x3 and 4096x3x3 slower)
    MARLNAV_SPLIT_VARIANT(3, 8, 8, false),
    MARLNAV_SPLIT_VARIANT(3, 3, 8, false),
};
#ifndef MARLNAV_SPLIT_TINY_WAVES
#define MARLNAV_SPLIT_TINY_WAVES 256  // (A/B builds)
#endif
constexpr int64_t kSplitTinyWaves = MARLNAV_SPLIT_TINY_WAVES;
// kSplitOwn (a finished env re-initialised by its own wave) for grids of at
// most two waves per SIMD (one env per wave): same box, graph replay,
// steady (profiles/r05_ab_tail_own2.txt, r05_ab_tail_ablate.txt): 512x16x32
// 7.98 -> 7.44 us, 1024x16x32 8.28 -> 7.58, 2048x16x32 9.27 -> 8.48;
// 4096x16x32 (four waves per SIMD) 11.59-11.62 -> 11.65-11.67. With the
// one-correction division its register allocation spilled SGPRs into the
// observation's hot blocks (2048: 9.96 us); with its parameters held in
// VGPRs (MARLNAV_OWN_VPIN, kernel_split.h) 8.24 us, 1024 7.44, 512 7.28
// against 9.14 / 7.93 / 7.78 for the default kernel (profiles/r05_ab_vpin.txt)
constexpr int64_t kSplitOwnMaxEnvs = MARLNAV_SPLIT_OWN_MAX;
#undef MARLNAV_SPLIT_VARIANT

// one-lane-per-row grids below kSplitBelowWaves * (pairs per row / 6) waves
// leave most SIMDs idle. A3/O8 (11 pairs): split below 587 wave tiles, i.e.
// about 11700 envs (round 5, graph replay, scripts/diag/family_ab.py,
// profiles/r05_family_ab.txt: 10240x3x8 split 6.17 vs block 6.46 us, 12288
// 6.67 vs 6.50, 16384 7.35 vs 6.51; round 2 had split faster at 16384)
constexpr int64_t kSplitBelowWaves = 320;
// ... except that with at most 6 pairs per row (A3/O3) the env-block kernel is
// faster from one full block of 64 envs on (graph replay, round 2, with
// kernarg preload: 64x3x3 4.20 vs 4.28 us, 1024x3x3 5.23 vs 5.37, 4096x3x3
// 5.41 vs 5.59, 8192x3x3 5.51 vs 6.10; 32x3x3 4.05 vs 5.05 stays split;
// profiles/r02_family_ab.txt)
constexpr int64_t kBlockFromEnvs = 64;

const SplitVariant *select_split(const MarlnavDims *d, const MarlnavStepBuffers &b, bool obs_only,
                                 bool force_size = false)
{
    if (d->obstacle_stride != d->num_obstacles) return nullptr;
    const SplitVariant *v = nullptr;
    for (const SplitVariant &x : kSplitVariants) {
        if (x.A != d->num_agents || x.O != d->num_obstacles) continue;
        if (x.lpr == 8) {  // the tiny-grid form: LPR=4 would leave >3/4 of the SIMDs idle
            const int64_t e4 = 64 / 4 / x.A;
            if ((d->num_parallel + e4 - 1) / e4 > kSplitTinyWaves) continue;
        }
        v = &x;  // the last applicable variant wins
    }
    if (!v) return nullptr;
    const int64_t row_waves = (d->num_parallel + tile_envs(v->A) - 1) / tile_envs(v->A);
    const int64_t pairs = 1 + v->O + (v->A - 1);
    if (!v->always && !force_size && row_waves * 6 >= kSplitBelowWaves * pairs)
        return nullptr;
    if (!v->always && !force_size && pairs <= 6 && d->num_parallel >= kBlockFromEnvs)
        return nullptr;
    if (!aligned(b.states, 16) || !aligned(b.obstacles, 16) || !aligned(b.target, 16) ||
        !aligned(b.obs, 16) || (b.states_out && !aligned(b.states_out, 16)))
        return nullptr;
    if (!obs_only && !aligned(b.actions, 16)) return nullptr;
    return v;
}

int launch_split(const SplitVariant &v, BlockFn fn, const StepArgs &args, const MarlnavParams &pr,
                 void *stream, const char *what)
{
    KArgs ka;
    ka.a = args;
    ka.p = pr;
    ka.a.W = v.epw;
    ka.a.ntiles = (args.P + v.epw - 1) / v.epw;
    const int64_t blocks = (ka.a.ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
    float *h_states = args.b.states;
    const float *h_actions = args.b.actions, *h_obstacles = args.b.obstacles,
                *h_target = args.b.target, *h_step_num = args.b.step_num;
    const uint8_t *h_terminates = args.b.terminates;
    int64_t h_P = args.P;
    void *kargs[] = {&h_states, &h_actions, &h_obstacles, &h_target, &h_step_num, &h_terminates,
                     &h_P, &ka};
    hipError_t e = hipLaunchKernel(reinterpret_cast<const void *>(fn), dim3((unsigned)blocks),
                                   dim3(64 * kWavesPerBlock), kargs, v.lds, (hipStream_t)stream);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return fail(MARLNAV_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
    return 0;
}

// env-block kernels (block_kernel) for these shapes
struct BlockVariant {
    int A, O;
    BlockFn step, obs, noisy;
    size_t lds;
    BlockFn step_draw;  // (or null) the step with a draw wave: grids of at most one block per CU
    int E;              // envs per block
};

// compute units of the current device (the draw-wave rule: at most one
// block per CU), read once per device
int device_cus()
{
    static std::atomic<int> cached[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int n = cached[dev].load(std::memory_order_relaxed);
    if (n <= 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n <= 0)
            n = 256;  // MI355X
        cached[dev].store(n, std::memory_order_relaxed);
    }
    return n;
}

// The draw-wave instantiation (block_kernel HELP): the native re-init's
// fresh-obstacle draws move from the agent waves' stage to a fourth wave on
// the SIMD a one-block-per-CU grid leaves idle (O draws per lane: O <= 3)
template <int A, int O>
constexpr BlockFn block_draw_fn()
{
    if constexpr (O <= 3 && MARLNAV_DRAW_WAVE) return block_kernel<A, O, false, false, true>;
    else return nullptr;
}

#define MARLNAV_BLOCK_VARIANT(A, O)                                                    \
    {A, O, block_kernel<A, O, false, false>, block_kernel<A, O, true, false>,          \
     block_kernel<A, O, false, true>, (size_t)BlockPlan<A, O>::FLOATS * 4,             \
     block_draw_fn<A, O>(), BlockPlan<A, O>::E}
const BlockVariant kBlockVariants[] = {
    MARLNAV_BLOCK_VARIANT(3, 3),
    MARLNAV_BLOCK_VARIANT(3, 8),
    MARLNAV_BLOCK_VARIANT(3, 1),
    MARLNAV_BLOCK_VARIANT(2, 1),
};
#undef MARLNAV_BLOCK_VARIANT

const BlockVariant *select_block(const MarlnavDims *d, const MarlnavStepBuffers &b, bool obs_only)
{
    if (d->obstacle_stride != d->num_obstacles) return nullptr;
    const BlockVariant *v = nullptr;
    for (const BlockVariant &x : kBlockVariants)
        if (x.A == d->num_agents && x.O == d->num_obstacles) v = &x;
    if (!v) return nullptr;
    if (!aligned(b.states, 16) || !aligned(b.obstacles, 16) || !aligned(b.target, 16) ||
        !aligned(b.obs, 16) || (b.states_out && !aligned(b.states_out, 16)))
        return nullptr;
    if (!obs_only && (!aligned(b.actions, 16) || !aligned(b.step_num, 16) ||
                      !aligned(b.terminates, 16) || (b.formation && !aligned(b.formation, 16))))
        return nullptr;
    return v;
}

int launch_block(const BlockVariant &v, BlockFn fn, const StepArgs &args, const MarlnavParams &pr,
                 void *stream, const char *what, int waves = 0)
{
    KArgs ka;
    ka.a = args;
    ka.p = pr;
    ka.a.W = v.E;
    ka.a.ntiles = (args.P + ka.a.W - 1) / ka.a.W;
    // the leading arguments (kHotKargsOff, kernel_args.h): staging pointers, P
    float *h_states = args.b.states;
    const float *h_actions = args.b.actions, *h_obstacles = args.b.obstacles,
                *h_target = args.b.target, *h_step_num = args.b.step_num;
    const uint8_t *h_terminates = args.b.terminates;
    int64_t h_P = args.P;
    void *kargs[] = {&h_states, &h_actions, &h_obstacles, &h_target, &h_step_num, &h_terminates,
                     &h_P, &ka};
    hipError_t e = hipLaunchKernel(reinterpret_cast<const void *>(fn), dim3((unsigned)ka.a.ntiles),
                                   dim3(64 * (waves ? waves : v.A)), kargs, v.lds, (hipStream_t)stream);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return fail(MARLNAV_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
    return 0;
}

bool has_variant(int A, int O)
{
    for (const KernelPair &k : kVariants)
        if (k.A == A && k.O == O) return true;
    return false;
}

KernelPair select_kernels(int A, int O)
{
    for (const KernelPair &k : kVariants)
        if (k.A == A && k.O == O) return k;
    return KernelPair{0, 0, wave_kernel<0, 0, false>, wave_kernel<0, 0, true>,
                      wave_kernel<0, 0, false, true>};
}

StepArgs make_args(const MarlnavDims *d, const Launch &L)
{
    StepArgs a;
    memset(&a, 0, sizeof(a));
    a.P = d->num_parallel;
    a.env_offset = d->env_offset;
    a.ntiles = L.ntiles;
    a.waves = L.waves;
    a.W = L.W;
    a.A = d->num_agents;
    a.O = d->num_obstacles;
    a.S = d->obstacle_stride;
    return a;
}

int launch(StepFn fn, const Launch &L, StepArgs args, MarlnavParams pr, void *stream,
           const char *what)
{
    void *kargs[] = {&args, &pr};
    const size_t lds = (size_t)L.plan.floats * 4 * kWavesPerBlock;
    hipError_t e = hipLaunchKernel(reinterpret_cast<const void *>(fn), dim3((unsigned)L.blocks),
                                   dim3(64 * kWavesPerBlock), kargs, lds, (hipStream_t)stream);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return fail(MARLNAV_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
    return 0;
}

// marlnav_debug_force_family / marlnav_debug_last_family (testing hooks)
// (a testing hook: atomic, so a test thread forcing a family never races a
// stepping thread's read)
std::atomic<int> g_family{MARLNAV_FAMILY_AUTO};
thread_local int g_last_family = MARLNAV_FAMILY_AUTO;

bool family_allowed(int f)
{
    const int g = g_family.load(std::memory_order_relaxed);
    return g == MARLNAV_FAMILY_AUTO || g == f;
}

}  // namespace

extern "C" {

int marlnav_abi_version(void) { return MARLNAV_ABI_VERSION; }

int marlnav_debug_force_family(int family)
{
    const int prev = g_family.load(std::memory_order_relaxed);
    if (family < MARLNAV_FAMILY_AUTO || family > MARLNAV_FAMILY_WAVE)
        return fail(MARLNAV_EINVAL, "unknown kernel family %d", family);
    g_family.store(family, std::memory_order_relaxed);
    return prev;
}

int marlnav_debug_last_family(void) { return g_last_family; }

#if MARLNAV_STAMPS
int marlnav_debug_stamps(void *buf)
{
    const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf));
    return e == hipSuccess ? 0 : fail(MARLNAV_ELAUNCH, "stamps: %s", hipGetErrorString(e));
}
#endif

int marlnav_debug_acos_range(uint32_t first, int64_t n, float *out, void *stream)
{
    if (n < 0 || (n > 0 && !out)) return fail(MARLNAV_EINVAL, "acos range: n < 0 or out NULL");
    if (n == 0) return 0;
    hipLaunchKernelGGL(acos_range_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, first, n, out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(MARLNAV_ELAUNCH, "acos range: %s", hipGetErrorString(e));
}

int marlnav_debug_fastdiv_check(uint32_t d_first, uint32_t d_stride, uint32_t nd, uint64_t *out,
                                void *stream)
{
    if (nd > 0 && !out) return fail(MARLNAV_EINVAL, "fastdiv check: out NULL");
    if (nd == 0) return 0;
    hipLaunchKernelGGL(fastdiv_check_kernel, dim3(nd), dim3(256), 0, (hipStream_t)stream, d_first,
                       d_stride, reinterpret_cast<unsigned long long *>(out));
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(MARLNAV_ELAUNCH, "fastdiv check: %s", hipGetErrorString(e));
}

const char *marlnav_last_error(void) { return g_err; }

int64_t marlnav_counter_slots(const MarlnavDims *d)
{
    if (validate(d)) return -1;
    return plan_launch(d).waves;
}

namespace {
// Parameter ranges under which the reward terms' divisions by bond_sharpness,
// init_dist and max_at_prop_d (div_c) and the bond reciprocal (recip_fast)
// are exact for every FAST-range distance: divisors in [2^-20, 2^20] (the
// sharpness in [2^-5, 2^20], so |(d - ideal) / sharpness| <= 2^48 and
// 1 + sd^2 <= 2^96), ideal_dist zero or in [2^-40, 2^40] (so d - ideal is
// zero or >= 2^-66 in magnitude).
bool terms_fast_params(const MarlnavParams &p)
{
    const auto in = [](float c, float lo, float hi) {
        const float a = fabsf(c);
        return a >= lo && a <= hi;
    };
    return in(p.bond_sharpness, 0x1p-5f, 0x1p20f) && in(p.init_dist, 0x1p-20f, 0x1p20f) &&
           in(p.max_at_prop_d, 0x1p-20f, 0x1p20f) &&
           (p.ideal_dist == 0.0f || in(p.ideal_dist, 0x1p-40f, 0x1p40f));
}
}  // namespace

int marlnav_step(const MarlnavDims *d, const MarlnavParams *pr_in, const MarlnavStepBuffers *b,
                 uint64_t step_idx, void *stream)
{
    if (!pr_in) return fail(MARLNAV_EINVAL, "params/buffers is NULL");
    MarlnavParams prm = *pr_in;
    prm.seed = native_seed_mix(prm.seed);  // the kernels key the native stream by the mixed seed
    prm.flags &= ~(kTermsFastFlag | kWriteThroughFlag);
    if (terms_fast_params(prm)) prm.flags |= kTermsFastFlag;
    const MarlnavParams *pr = &prm;
    if (int rc = validate(d)) return rc;
    // written-through outputs (device_math.h kWriteThroughFlag) for launches
    // that write at least kWriteThroughMinBytes
    {
        const int64_t A = d->num_agents, D = obs_dim(d->num_agents, d->num_obstacles);
        const int64_t wbytes = (int64_t)d->num_parallel * (20 * A + 4 * A * D + 11);
        if (wbytes >= kWriteThroughMinBytes) prm.flags |= kWriteThroughFlag;
    }
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
    const Launch L = plan_launch(d);
    StepArgs args = make_args(d, L);
    args.b = *b;
    args.step_idx = step_idx;
    if (!args.b.states_out) {
        args.b.states_out = args.b.states;  // in place
    } else if (args.b.states_out != args.b.states) {
        const size_t n = (size_t)d->num_parallel * d->num_agents * 5 * sizeof(float);
        const char *a0 = (const char *)args.b.states, *b0 = (const char *)args.b.states_out;
        if (a0 < b0 + n && b0 < a0 + n)
            return fail(MARLNAV_EINVAL, "states_out overlaps states");
    }
    const bool noisy = !b->fresh_states && (pr->flags & MARLNAV_NOISY_AGENTS);
    const bool fsplit = g_family.load(std::memory_order_relaxed) == MARLNAV_FAMILY_SPLIT;
    if (family_allowed(MARLNAV_FAMILY_SPLIT))
        if (const SplitVariant *v = select_split(d, args.b, false, fsplit)) {
            g_last_family = MARLNAV_FAMILY_SPLIT;
            const bool own = !noisy && v->step_own && d->num_parallel <= kSplitOwnMaxEnvs &&
                             !MARLNAV_SPLIT_OWN_OFF;
            return launch_split(*v, noisy ? v->noisy : (own ? v->step_own : v->step), args, *pr,
                                stream, "marlnav_step");
        }
    if (family_allowed(MARLNAV_FAMILY_BLOCK))
        if (const BlockVariant *v = select_block(d, args.b, false)) {
            g_last_family = MARLNAV_FAMILY_BLOCK;
            // one block per CU (MI355X: 256 CUs) leaves a SIMD of each CU idle
            const int64_t nblk = (d->num_parallel + v->E - 1) / v->E;
            if (!noisy && v->step_draw && nblk <= device_cus() && !b->fresh_states)
                return launch_block(*v, v->step_draw, args, *pr, stream, "marlnav_step", v->A + 1);
            return launch_block(*v, noisy ? v->noisy : v->step, args, *pr, stream, "marlnav_step");
        }
    const KernelPair k = select_kernels(d->num_agents, d->num_obstacles);
    g_last_family = MARLNAV_FAMILY_WAVE;
    return launch(noisy ? k.noisy : k.step, L, args, *pr, stream, "marlnav_step");
}

int marlnav_observe(const MarlnavDims *d, const MarlnavParams *params, const float *states,
                    const float *obstacles, const float *target, float *obs, void *stream)
{
    if (int rc = validate(d)) return rc;
    if (!states || !obstacles || !target || !obs)
        return fail(MARLNAV_EINVAL, "a required observe buffer is NULL");
    const Launch L = plan_launch(d);
    StepArgs args = make_args(d, L);
    args.b.states = const_cast<float *>(states);
    args.b.obstacles = const_cast<float *>(obstacles);
    args.b.target = const_cast<float *>(target);
    args.b.obs = obs;
    MarlnavParams pr;
    memset(&pr, 0, sizeof(pr));
    // the angle cap (environment.py:172-177) is the only parameter observe reads;
    // NULL params: the reference's default (environment.py:65)
    pr.cap_distance = params ? params->cap_distance : 0.1f;
    if ((int64_t)d->num_parallel * d->num_agents * obs_dim(d->num_agents, d->num_obstacles) * 4 >=
        kWriteThroughMinBytes)
        pr.flags |= kWriteThroughFlag;
    const bool fsplit = g_family.load(std::memory_order_relaxed) == MARLNAV_FAMILY_SPLIT;
    if (family_allowed(MARLNAV_FAMILY_SPLIT))
        if (const SplitVariant *v = select_split(d, args.b, true, fsplit)) {
            g_last_family = MARLNAV_FAMILY_SPLIT;
            return launch_split(*v, v->obs, args, pr, stream, "marlnav_observe");
        }
    if (family_allowed(MARLNAV_FAMILY_BLOCK))
        if (const BlockVariant *v = select_block(d, args.b, true)) {
            g_last_family = MARLNAV_FAMILY_BLOCK;
            return launch_block(*v, v->obs, args, pr, stream, "marlnav_observe");
        }
    g_last_family = MARLNAV_FAMILY_WAVE;
    return launch(select_kernels(d->num_agents, d->num_obstacles).obs, L, args, pr, stream,
                  "marlnav_observe");
}

int marlnav_reinit_all(const MarlnavDims *d, const MarlnavParams *pr, const float *formation,
                       float *states, float *obstacles, float *target, uint64_t step_idx,
                       void *stream)
{
    if (int rc = validate(d)) return rc;
    if (!pr || !formation || !states || !obstacles || !target)
        return fail(MARLNAV_EINVAL, "a required reinit buffer is NULL");
    const unsigned blocks = (unsigned)((d->num_parallel + 255) / 256);
    MarlnavParams prm = *pr;
    prm.seed = native_seed_mix(prm.seed);  // as marlnav_step
    hipLaunchKernelGGL(reinit_all_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       d->num_parallel, d->num_agents, d->obstacle_stride, d->env_offset,
                       step_idx, prm, formation, states, obstacles, target);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(MARLNAV_ELAUNCH, "marlnav_reinit_all: %s", hipGetErrorString(e));
    return 0;
}

int marlnav_formation_obs(const MarlnavDims *d, const float *formation, float *out,
                          void *stream)
{
    if (int rc = validate(d)) return rc;
    if (!formation || !out) return fail(MARLNAV_EINVAL, "formation/out is NULL");
    const int n = d->num_agents * d->num_agents;
    hipLaunchKernelGGL(formation_obs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d->num_agents, formation, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(MARLNAV_ELAUNCH, "marlnav_formation_obs: %s", hipGetErrorString(e));
    return 0;
}

int marlnav_counters_total(const MarlnavDims *d, const uint64_t *counters, uint64_t *out3,
                           void *stream)
{
    const int64_t slots = marlnav_counter_slots(d);
    if (slots < 0) return MARLNAV_EINVAL;
    if (!counters || !out3) return fail(MARLNAV_EINVAL, "counters/out3 is NULL");
    hipLaunchKernelGGL(counters_total_kernel, dim3(3), dim3(64), 0, (hipStream_t)stream,
                       counters, slots, out3);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(MARLNAV_ELAUNCH, "marlnav_counters_total: %s", hipGetErrorString(e));
    return 0;
}

}  // extern "C"
