// Exhaustive check of v_sqrt_f32 (__builtin_amdgcn_sqrtf) against the IEEE
// correctly rounded sqrtf (hipcc's sequence: v_sqrt + residual fix-up) over
// every positive finite float, and inside the FAST range [2^-96, 2^96] that
// sqrt_fast (device_math.h) guards. Prints mismatch counts and examples.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 sqrt_probe.hip -o sqrt_probe
// Also: the shipped sqrt_fast (marl-nav_amd/csrc/device_math.h) against
// IEEE sqrtf over every float of its range [2^-96, 2^96] and zero.
#include "../../marl-nav_amd/csrc/marlnav_step.hip"

__global__ void probe_fast(uint32_t base, unsigned long long *cnt, uint32_t *ex)
{
    const uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float(u);
    if (!((x >= 0x1p-96f && x <= 0x1p96f) || u == 0u)) return;
    bool ok = true;
    const float a = sqrt_fast(x, ok);
    const float b = __builtin_sqrtf(x);
    if (__float_as_uint(a) != __float_as_uint(b) || !ok) {
        const unsigned long long k = atomicAdd(cnt, 1ull);
        if (k < 8) ex[k] = u;
    }
}

__global__ void probe(uint32_t base, unsigned long long *cnt, unsigned long long *cnt_fast,
                      uint32_t *ex)
{
    const uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;
    if (u > 0x7f7fffffu) return;  // positive finite only
    const float x = __uint_as_float(u);
    const float a = __builtin_amdgcn_sqrtf(x);
    const float b = __builtin_sqrtf(x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
        const unsigned long long k = atomicAdd(cnt, 1ull);
        if (k < 8) ex[k] = u;
        if (x >= 0x1p-96f && x <= 0x1p96f) {
            atomicAdd(cnt_fast, 1ull);
            // direction inside the FAST range: v_sqrt above / below the
            // correctly rounded value, and by more than one ulp
            const int d = (int)__float_as_uint(a) - (int)__float_as_uint(b);
            atomicAdd(cnt_fast + (d > 0 ? 1 : 2), 1ull);
            if (d > 1 || d < -1) atomicAdd(cnt_fast + 3, 1ull);
        }
    }
}

int main()
{
    unsigned long long *cnt, *cf;
    uint32_t *ex;
    hipMalloc(&cnt, 8);
    hipMalloc(&cf, 32);
    hipMalloc(&ex, 32);
    hipMemset(cnt, 0, 8);
    hipMemset(cf, 0, 32);
    hipMemset(ex, 0, 32);
    const uint32_t chunk = 1u << 28;
    for (uint64_t b = 0; b <= 0x7f7fffffull; b += chunk)
        hipLaunchKernelGGL(probe, dim3(chunk / 256), dim3(256), 0, 0, (uint32_t)b, cnt, cf, ex);
    unsigned long long h = 0, hf = 0;
    uint32_t he[8];
    hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hf, cf, 8, hipMemcpyDeviceToHost);
    hipMemcpy(he, ex, 32, hipMemcpyDeviceToHost);
    unsigned long long hd[4];
    hipMemcpy(hd, cf, 32, hipMemcpyDeviceToHost);
    printf("v_sqrt_f32 != IEEE sqrtf: %llu of 2139095040 positive finite floats; %llu inside [2^-96, 2^96]"
           " (v_sqrt above: %llu, below: %llu, off by more than 1 ulp: %llu)\n", h, hf, hd[1], hd[2], hd[3]);
    for (int i = 0; i < 8 && i < (int)h; ++i) printf("  x bits 0x%08x (%g)\n", he[i], (double)__builtin_bit_cast(float, he[i]));
    unsigned long long *cq;
    uint32_t *eq;
    hipMalloc(&cq, 8);
    hipMalloc(&eq, 32);
    hipMemset(cq, 0, 8);
    for (uint64_t b = 0; b <= 0x7f7fffffull; b += chunk)
        hipLaunchKernelGGL(probe_fast, dim3(chunk / 256), dim3(256), 0, 0, (uint32_t)b, cq, eq);
    unsigned long long hq = 0;
    uint32_t heq[8];
    hipMemcpy(&hq, cq, 8, hipMemcpyDeviceToHost);
    hipMemcpy(heq, eq, 32, hipMemcpyDeviceToHost);
    printf("sqrt_fast != IEEE sqrtf: %llu floats of [2^-96, 2^96] and +0\n", hq);
    for (int i = 0; i < 8 && i < (int)hq; ++i) printf("  x bits 0x%08x\n", heq[i]);
    printf("hip: %s\n", hipGetErrorString(hipDeviceSynchronize()));
    return hq == 0 ? 0 : 1;
}
