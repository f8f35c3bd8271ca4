// Dispatch / launch-overhead probe: how long does the GPU take to start all
// waves of a grid, and what does an empty kernel cost, for the grid shapes
// the step kernel uses. Build: hipcc --offload-arch=gfx950 -O3 dispatch_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

struct Big { float f[40]; void *p[18]; long long l[6]; };

__global__ void probe(unsigned long long *t, int nwaves_per_block, Big big)
{
    extern __shared__ float lds[];
    const unsigned long long now = wall_clock64();
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * nwaves_per_block + (threadIdx.x >> 6);
        t[2 * w] = now;
        t[2 * w + 1] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
    }
    if (big.f[0] == 12345.0f) lds[threadIdx.x] = big.f[threadIdx.x % 40];
}

int main()
{
    unsigned long long *t;
    hipMalloc(&t, sizeof(unsigned long long) * 2 * 200000);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    Big big{};
    const int shapes[][3] = {{205, 256, 0}, {820, 256, 0}, {820, 256, 23000}, {1024, 192, 17800},
                             {3280, 64, 0}, {26215, 256, 23000}, {4096, 256, 0}};
    for (auto &s : shapes) {
        const int blocks = s[0], threads = s[1], lds = s[2];
        const int wpb = threads / 64;
        std::vector<float> ms;
        std::vector<double> spread;
        for (int rep = 0; rep < 20; ++rep) {
            hipMemset(t, 0, sizeof(unsigned long long) * 2 * blocks * wpb);
            hipDeviceSynchronize();
            hipEventRecord(a, 0);
            hipLaunchKernelGGL(probe, dim3(blocks), dim3(threads), lds, 0, t, wpb, big);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float x;
            hipEventElapsedTime(&x, a, b);
            ms.push_back(x * 1000.0f);
            std::vector<unsigned long long> h(2 * blocks * wpb);
            hipMemcpy(h.data(), t, h.size() * 8, hipMemcpyDeviceToHost);
            unsigned long long lo = ~0ull, hi = 0;
            unsigned long long xlo[16], xhi[16];
            for (int x = 0; x < 16; ++x) { xlo[x] = ~0ull; xhi[x] = 0; }
            for (int w = 0; w < blocks * wpb; ++w) {
                lo = std::min(lo, h[2 * w]);
                hi = std::max(hi, h[2 * w]);
                const int x = (int)(h[2 * w + 1] & 15);
                xlo[x] = std::min(xlo[x], h[2 * w]);
                xhi[x] = std::max(xhi[x], h[2 * w]);
            }
            spread.push_back((hi - lo) * 0.01);  // 100 MHz -> us
            if (rep == 19) {
                printf("   per-xcc first/last entry (us):");
                for (int x = 0; x < 16; ++x)
                    if (xhi[x]) printf(" %d:%.2f/%.2f", x, (xlo[x] - lo) * 0.01, (xhi[x] - lo) * 0.01);
                printf("\n");
            }
        }
        std::sort(ms.begin(), ms.end());
        std::sort(spread.begin(), spread.end());
        printf("blocks=%6d threads=%4d lds=%6d waves=%7d  event_us median %.2f  start_spread_us median %.2f\n",
               blocks, threads, lds, blocks * wpb, ms[ms.size() / 2], spread[spread.size() / 2]);
    }
    return 0;
}
