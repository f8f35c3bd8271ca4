// Floor probes for the A3/O3 step at 65,536 envs (scripts/probes/floor.py):
// kernels with the block kernel's grid (one 192-thread workgroup per 64 envs)
// that move exactly the step's bytes (read 121 B, write 215 B per env) with
// no arithmetic, optionally with a dependent VALU chain of `chain` steps
// per lane between the stage and the stores. Timing only; never loaded by
// the package.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
typedef __attribute__((address_space(3))) void LdsVoid;
typedef float v4f_t __attribute__((ext_vector_type(4)));

struct Spans {
    const float *states, *actions, *obstacles, *target, *step_num;
    const uint8_t *terminates;
    float *obs, *states_out, *reward, *step_out;
    uint8_t *terminated, *truncated, *terminates_out;
};

template <int NB>
__device__ __forceinline__ void glds(const void *src, float *dst, unsigned lane)
{
    constexpr int N16 = NB / 16, R4 = (NB % 16) / 4;
#pragma unroll
    for (int k = 0; k * 64 < N16; ++k) {
        const char *s = reinterpret_cast<const char *>(src) + k * 1024;
        if ((k + 1) * 64 <= N16 || (int)lane < N16 - k * 64)
            __builtin_amdgcn_global_load_lds(s + lane * 16u, (LdsVoid *)(dst + k * 256), 16, 0, 0);
    }
    if constexpr (R4 > 0) {
        const char *s = reinterpret_cast<const char *>(src) + N16 * 16;
        if ((int)lane < R4)
            __builtin_amdgcn_global_load_lds(s + lane * 4u, (LdsVoid *)(dst + N16 * 4), 4, 0, 0);
    }
}

constexpr int E = 64, A = 3, D = 12, R = E * A;
constexpr int L_ST = 0, L_ACT = L_ST + R * 5, L_OB = L_ACT + R * 2, L_TG = L_OB + E * 6,
              L_SN = L_TG + E * 2, L_TM = L_SN + E, L_OBS = L_TM + E / 4, L_END = L_OBS + R * D;

template <bool NT>
__device__ __forceinline__ void st4(float *p, float4 v)
{
    if (NT)
        __builtin_nontemporal_store(v4f_t{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f_t *>(p));
    else
        *reinterpret_cast<float4 *>(p) = v;
}

template <bool NT>
__global__ void __launch_bounds__(192) k_stage_store(Spans s, int chain)
{
    __shared__ __attribute__((aligned(16))) float lds[L_END + 4];
    const int tid = threadIdx.x, w = tid >> 6;
    const unsigned lane = tid & 63;
    const int64_t e0 = (int64_t)blockIdx.x * E;
    if (w == 0) {
        glds<R * 20>(s.states + e0 * 15, lds + L_ST, lane);
        glds<E * 8>(s.target + e0 * 2, lds + L_TG, lane);
    } else if (w == 1) {
        glds<R * 8>(s.actions + e0 * 6, lds + L_ACT, lane);
        glds<E * 4>(s.step_num + e0, lds + L_SN, lane);
    } else {
        glds<E * 24>(s.obstacles + e0 * 6, lds + L_OB, lane);
        glds<E>(s.terminates + e0, lds + L_TM, lane);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // a row's worth of LDS reads and a dependent chain per lane
    const int r = (int)lane * A + w;
    float x = lds[L_ST + 5 * r] + lds[L_ACT + 2 * r] + lds[L_OB + 6 * lane + w];
    for (int i = 0; i < chain; ++i) x = __builtin_fmaf(x, 0.999f, 1.0f);
    float *row = lds + L_OBS + r * D;
#pragma unroll
    for (int k = 0; k < D; ++k) row[k] = x + k;
    __syncthreads();
    if (w == 0) {
        const int64_t e = e0 + lane;
        s.reward[e] = x;
        s.terminated[e] = (uint8_t)(x > 5.0f);
        s.truncated[e] = (uint8_t)(x > 6.0f);
        s.terminates_out[e] = (uint8_t)(x > 7.0f);
        s.step_out[e] = lds[L_SN + lane] + 1.0f;
    }
    // rows (R*D floats) and states (R*5) out, 16-byte stores, all reads first
    constexpr int Q1 = R * D / 4, Q2 = R * 5 / 4;
    float4 v1[(Q1 + 191) / 192], v2[(Q2 + 191) / 192];
#pragma unroll
    for (int k = 0; k < (Q1 + 191) / 192; ++k)
        if (tid + k * 192 < Q1) v1[k] = reinterpret_cast<const float4 *>(lds + L_OBS)[tid + k * 192];
#pragma unroll
    for (int k = 0; k < (Q2 + 191) / 192; ++k)
        if (tid + k * 192 < Q2) v2[k] = reinterpret_cast<const float4 *>(lds + L_ST)[tid + k * 192];
#pragma unroll
    for (int k = 0; k < (Q1 + 191) / 192; ++k)
        if (tid + k * 192 < Q1) st4<NT>(s.obs + e0 * (A * D) + 4 * (tid + k * 192), v1[k]);
#pragma unroll
    for (int k = 0; k < (Q2 + 191) / 192; ++k)
        if (tid + k * 192 < Q2) st4<NT>(s.states_out + e0 * 15 + 4 * (tid + k * 192), v2[k]);
}

__global__ void __launch_bounds__(192) k_empty(float *p)
{
    if (p && threadIdx.x == 1000) p[0] = 1.0f;
}
}  // namespace

extern "C" int floor_launch(int which, int blocks, void *spans, int chain, void *stream)
{
    const Spans &s = *reinterpret_cast<const Spans *>(spans);
    hipError_t e;
    if (which == 0) {
        hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(192), 0, (hipStream_t)stream, nullptr);
    } else if (which == 1) {
        hipLaunchKernelGGL(k_stage_store<true>, dim3(blocks), dim3(192), 0, (hipStream_t)stream, s,
                           chain);
    } else {
        hipLaunchKernelGGL(k_stage_store<false>, dim3(blocks), dim3(192), 0, (hipStream_t)stream, s,
                           chain);
    }
    e = hipGetLastError();
    return (int)e;
}
