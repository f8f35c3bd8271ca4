// Instruction-fetch probe: the same VALU instruction count as straight-line
// code (cold in the instruction cache at every launch) vs a short loop body
// (fetched once). 1 and 3 waves per SIMD, timed with events over launches.
// Build: hipcc --offload-arch=gfx950 -O3 ifetch_probe.hip -o ifetch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x
#define BODY "v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4\n"

__global__ void __launch_bounds__(64) straight(float *out, float k)
{
    float a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
    // 8192 instructions of straight-line code (~64 KiB... 4 B each = 32 KiB)
    asm volatile(".rept 2048\n" BODY ".endr\n" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(k));
    out[blockIdx.x * 64 + threadIdx.x] = a + b + c + d;
}

__global__ void __launch_bounds__(64) looped(float *out, float k, int iters)
{
    float a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
    for (int i = 0; i < iters; ++i)  // 256-instruction body (1 KiB)
        asm volatile(".rept 64\n" BODY ".endr\n" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(k));
    out[blockIdx.x * 64 + threadIdx.x] = a + b + c + d;
}

__global__ void __launch_bounds__(64) empty(float *out) { if (out == nullptr) out[0] = 0; }

int main()
{
    float *out;
    hipMalloc(&out, 64 * 4096 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int blocks : {1024, 3072}) {
        for (int kind = 0; kind < 3; ++kind) {
            for (int w = 0; w < 3; ++w) {  // warm-up
                if (kind == 0) straight<<<blocks, 64>>>(out, 1.0f);
                else if (kind == 1) looped<<<blocks, 64>>>(out, 1.0f, 32);
                else empty<<<blocks, 64>>>(out);
            }
            hipEventRecord(e0);
            const int n = 50;
            for (int r = 0; r < n; ++r) {
                if (kind == 0) straight<<<blocks, 64>>>(out, 1.0f);
                else if (kind == 1) looped<<<blocks, 64>>>(out, 1.0f, 32);
                else empty<<<blocks, 64>>>(out);
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("blocks %d %s: %.2f us per launch\n", blocks,
                   kind == 0 ? "straight 8192 instr" : (kind == 1 ? "loop 32x256 instr" : "empty"),
                   ms * 1000.0f / n);
        }
    }
    return 0;
}
