// kernarg_probe.hip - per-launch GPU time of a fixed-length kernel against its
// kernel-argument size and launch mode (stream launches in a tight host loop
// vs one hipGraph of the same launches), to separate the runtime's per-launch
// dispatch cost from the step kernel's own time (profiles/r06_launch_modes.txt).
// The kernel sleeps `iters` x s_sleep 127 (~3.5 us each) per wave so the GPU, not the host,
// sets the pace; 256 workgroups of 64 threads (configs[4]'s one block per CU).
// Build: hipcc -O2 --offload-arch=gfx950 kernarg_probe.hip -o kernarg_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int NB>
struct Blob {
    unsigned char b[NB];
};

template <int NB>
__global__ void spin_kernel(Blob<NB> arg, int iters, float *out)
{
    for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (float)arg.b[NB - 1];
}

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                              \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

template <int NB>
int run(hipStream_t s, float *out, int iters, int K)
{
    Blob<NB> a{};
    a.b[NB - 1] = 1;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // stream launches (warm-up first)
    for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(spin_kernel<NB>, dim3(256), dim3(64), 0, s, a, iters, out);
    CHECK(hipStreamSynchronize(s));
    float best_s = 1e30f, best_g = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < K; ++i) hipLaunchKernelGGL(spin_kernel<NB>, dim3(256), dim3(64), 0, s, a, iters, out);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best_s = ms * 1e3f / K < best_s ? ms * 1e3f / K : best_s;
    }
    // the same K launches captured in a graph, replayed
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(spin_kernel<NB>, dim3(256), dim3(64), 0, s, a, iters, out);
    CHECK(hipStreamEndCapture(s, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHECK(hipGraphLaunch(ge, s));
    CHECK(hipStreamSynchronize(s));
    for (int rep = 0; rep < 5; ++rep) {
        CHECK(hipEventRecord(e0, s));
        CHECK(hipGraphLaunch(ge, s));
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best_g = ms * 1e3f / K < best_g ? ms * 1e3f / K : best_g;
    }
    printf("kernarg %4d B  iters %3d  stream %.3f us/launch  graph %.3f us/launch  diff %+.3f\n", NB, iters,
           best_s, best_g, best_s - best_g);
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
    return 0;
}

int main()
{
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    float *out;
    if (hipMalloc(&out, 64) != hipSuccess) return 1;
    const int K = 400;
    for (int iters : {0, 1, 2}) {
        if (run<16>(s, out, iters, K)) return 1;
        if (run<64>(s, out, iters, K)) return 1;
        if (run<432>(s, out, iters, K)) return 1;
        if (run<1024>(s, out, iters, K)) return 1;
    }
    (void)hipFree(out);
    return 0;
}
