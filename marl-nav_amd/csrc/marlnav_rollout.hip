// marlnav_rollout.hip - gfx950 kernels for the rollout side of the training
// loop that drives Env.step: MAPPO._process_rewards (marlnav/models.py:131-148)
// as a device scan instead of a Python loop of T x 3 small tensor ops.
//
// Layout: rewards (T, P) fp32 and done (T, P) bool as stacked step rows; one
// thread per env walks its column backwards (coalesced across the wave), in
// float64 as the reference accumulates (torch.zeros(P, dtype=float)). Mean
// and unbiased std are two-pass block reductions in a fixed order, so results
// are deterministic run to run.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

#include "../../include/marlnav.h"

__attribute__((visibility("hidden"))) int marlnav_internal_fail(int code, const char *msg);

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ double block_sum(double v, double *sh)
{
    // wave partial sums (fixed shuffle tree), then the 4 waves in order
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int i = 0; i < kThreads / 64; ++i) t += sh[i];
    __syncthreads();
    return t;  // valid in thread 0
}

// G_t = done_t ? 0 : r_t + gamma * G_{t+1}  (models.py:133-137)
__global__ void __launch_bounds__(kThreads) returns_kernel(const float *__restrict__ rew,
                                                            const uint8_t *__restrict__ done,
                                                            int64_t T, int64_t P, double gamma,
                                                            double *__restrict__ ret,
                                                            double *__restrict__ partial)
{
    __shared__ double sh[kThreads / 64];
    const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    double s = 0.0;
    if (e < P) {
        double g = 0.0;
        for (int64_t t = T - 1; t >= 0; --t) {
            const int64_t i = t * P + e;
            g = done[i] ? 0.0 : (double)rew[i] + gamma * g;
            ret[i] = g;
            s += g;
        }
    }
    const double b = block_sum(s, sh);
    if (threadIdx.x == 0) partial[blockIdx.x] = b;
}

// sum of the block partials in index order -> out (one block)
__global__ void __launch_bounds__(kThreads) finish_kernel(const double *__restrict__ partial,
                                                           int64_t nb, int64_t n, int mode,
                                                           double *__restrict__ stats)
{
    __shared__ double sh[kThreads / 64];
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < nb; i += kThreads) s += partial[i];
    const double t = block_sum(s, sh);
    if (threadIdx.x == 0) {
        if (mode == 0)
            stats[0] = t / (double)n;                // mean
        else
            stats[1] = sqrt(t / (double)(n - 1));    // unbiased std
    }
}

__global__ void __launch_bounds__(kThreads) sqdev_kernel(const double *__restrict__ ret,
                                                          int64_t T, int64_t P,
                                                          const double *__restrict__ stats,
                                                          double *__restrict__ partial)
{
    __shared__ double sh[kThreads / 64];
    const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const double mean = stats[0];
    double s = 0.0;
    if (e < P)
        for (int64_t t = T - 1; t >= 0; --t) {
            const double d = ret[t * P + e] - mean;
            s += d * d;
        }
    const double b = block_sum(s, sh);
    if (threadIdx.x == 0) partial[blockIdx.x] = b;
}

// (G - mean) / (std + 1e-12)  (models.py:143-144)
__global__ void __launch_bounds__(kThreads) normalize_kernel(double *__restrict__ ret, int64_t T,
                                                              int64_t P,
                                                              const double *__restrict__ stats)
{
    const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (e >= P) return;
    const double mean = stats[0], den = stats[1] + 1e-12;
    for (int64_t t = 0; t < T; ++t) {
        const int64_t i = t * P + e;
        ret[i] = (ret[i] - mean) / den;
    }
}

int64_t blocks_for(int64_t P) { return (P + kThreads - 1) / kThreads; }

}  // namespace

extern "C" {

int64_t marlnav_returns_work_size(int64_t P)
{
    return P < 1 ? -1 : 2 * blocks_for(P);
}

int marlnav_discounted_returns(const float *rewards, const uint8_t *done, int64_t T, int64_t P,
                               double gamma, double *returns, double *stats, double *work,
                               void *stream)
{
    if (T < 1 || P < 1) return marlnav_internal_fail(MARLNAV_EINVAL, "T and P must be >= 1");
    if (!rewards || !done || !returns || !stats || !work)
        return marlnav_internal_fail(MARLNAV_EINVAL, "a required returns buffer is NULL");
    const int64_t nb = blocks_for(P);
    if (nb > 0x7fffffff) return marlnav_internal_fail(MARLNAV_EINVAL, "P too large");
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)nb), blk(kThreads);
    hipLaunchKernelGGL(returns_kernel, grid, blk, 0, s, rewards, done, T, P, gamma, returns, work);
    hipLaunchKernelGGL(finish_kernel, dim3(1), blk, 0, s, work, nb, T * P, 0, stats);
    hipLaunchKernelGGL(sqdev_kernel, grid, blk, 0, s, returns, T, P, stats, work + nb);
    hipLaunchKernelGGL(finish_kernel, dim3(1), blk, 0, s, work + nb, nb, T * P, 1, stats);
    hipLaunchKernelGGL(normalize_kernel, grid, blk, 0, s, returns, T, P, stats);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return marlnav_internal_fail(MARLNAV_ELAUNCH, hipGetErrorString(e));
    return 0;
}

}  // extern "C"
