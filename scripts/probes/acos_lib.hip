// The device library's acosf exactly as the step kernels get it (same
// compiler flags as marl-nav_amd/csrc/Makefile), over consecutive fp32 bit
// patterns, behind a C entry point for tests/golden/acos_dev_check.py.
// Build: make -C scripts/probes libacos.so (on the host; the .so travels).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void acos_range_kernel(uint32_t first, int64_t n, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = acosf(__uint_as_float(first + (uint32_t)i));
}

extern "C" int acos_dev_range(uint32_t first, int64_t n, void *out, void *stream)
{
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(acos_range_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, first,
                       n, (float *)out);
    return (int)hipGetLastError();
}

// v_sqrt_f32 (the instruction inside the library's acosf) of r = k * 2^-25
// for k in [k0, k0 + n): every r the acosf's |x| > 0.5 branch can feed it
// (r = 0.5 - 0.5|x| with |x| in (0.5, 1] a multiple of 2^-24)
__global__ void vsqrt_grid_kernel(uint32_t k0, int64_t n, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = __builtin_amdgcn_sqrtf((float)(k0 + (uint32_t)i) * 0x1.0p-25f);
}

extern "C" int vsqrt_grid(uint32_t k0, int64_t n, void *out, void *stream)
{
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(vsqrt_grid_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, k0, n,
                       (float *)out);
    return (int)hipGetLastError();
}
