// step_loop - a C++ host of libmarlnav.so that uses nothing but the C ABI
// (include/marlnav.h) and the HIP runtime: no Python, no torch. It is what a
// C/C++ rollout driver replacing the reference's Python Env.step loop
// (marlnav/environment.py:92-107, driven by MAPPO.get_data, models.py:106-129)
// would do: allocate the env buffers on the device, initialise them natively
// (marlnav_reinit_all, the Env.__init__ sampler call environment.py:26-30),
// observe the fresh-env formation once (marlnav_formation_obs), then call
// marlnav_step once per step with that step's actions and read the episode
// counters (marlnav_counters_total).
//
//   step_loop <in.bin> <out.bin>
// in.bin:  MarlnavDims | MarlnavParams | int32 steps | float formation[5A+2] |
//          float actions[steps][P][A][2]   (raw little-endian structs)
// out.bin: states | obstacles | target | step_num | terminates (u8) | obs of
//          the last step | reward | terminated (u8) | truncated (u8) |
//          uint64 counters[3]
// tests/test_gpu_parity.py::test_c_host_matches_python_env runs it against
// the Python Env on the same inputs.
//
// Build (examples/c_host/Makefile):
//   hipcc -O2 -std=c++17 step_loop.cpp -I../../include -L../../marl-nav_amd/lib -lmarlnav
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "marlnav.h"

namespace {

void die(const char *what)
{
    std::fprintf(stderr, "step_loop: %s\n", what);
    std::exit(1);
}

void check_hip(hipError_t e, const char *what)
{
    if (e != hipSuccess) {
        std::fprintf(stderr, "step_loop: %s: %s\n", what, hipGetErrorString(e));
        std::exit(1);
    }
}

void check_rc(int rc, const char *what)
{
    if (rc != 0) {
        std::fprintf(stderr, "step_loop: %s failed (%d): %s\n", what, rc, marlnav_last_error());
        std::exit(1);
    }
}

template <class T>
T *dev_alloc(size_t n)
{
    void *p = nullptr;
    check_hip(hipMalloc(&p, n * sizeof(T) + 16), "hipMalloc");
    check_hip(hipMemset(p, 0, n * sizeof(T) + 16), "hipMemset");
    return static_cast<T *>(p);
}

template <class T>
void get(std::FILE *f, T *dst, size_t n)
{
    if (std::fread(dst, sizeof(T), n, f) != n) die("short input file");
}

template <class T>
void put(std::FILE *f, const T *dev, size_t n)
{
    std::vector<T> h(n);
    check_hip(hipMemcpy(h.data(), dev, n * sizeof(T), hipMemcpyDeviceToHost), "hipMemcpy D2H");
    if (std::fwrite(h.data(), sizeof(T), n, f) != n) die("short write");
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc != 3) die("usage: step_loop <in.bin> <out.bin>");
    if (marlnav_abi_version() != MARLNAV_ABI_VERSION) die("libmarlnav ABI version mismatch");
    std::FILE *in = std::fopen(argv[1], "rb");
    if (!in) die("cannot open input");
    MarlnavDims dims;
    MarlnavParams params;
    int32_t steps = 0;
    get(in, &dims, 1);
    get(in, &params, 1);
    get(in, &steps, 1);
    const int64_t P = dims.num_parallel;
    const int A = dims.num_agents, O = dims.num_obstacles, S = dims.obstacle_stride;
    const int D = 2 + 2 * O + 2 * (A - 1);
    std::vector<float> form(5 * A + 2), acts((size_t)steps * P * A * 2);
    get(in, form.data(), form.size());
    get(in, acts.data(), acts.size());
    std::fclose(in);

    hipStream_t stream;
    check_hip(hipStreamCreate(&stream), "hipStreamCreate");
    const int64_t slots = marlnav_counter_slots(&dims);
    if (slots <= 0) die("marlnav_counter_slots");

    MarlnavStepBuffers b = {};
    b.states = dev_alloc<float>(P * A * 5);
    b.obstacles = dev_alloc<float>(P * S * 2);
    b.target = dev_alloc<float>(P * 2);
    b.step_num = dev_alloc<float>(P);
    b.terminates = dev_alloc<uint8_t>(P);
    float *actions = dev_alloc<float>(P * A * 2);
    b.actions = actions;
    float *formation = dev_alloc<float>(form.size());
    b.formation = formation;
    float *formation_obs = dev_alloc<float>(2 * A * A);
    b.formation_obs = formation_obs;
    b.obs = dev_alloc<float>(P * A * D);
    b.reward = dev_alloc<float>(P);
    b.terminated = dev_alloc<uint8_t>(P);
    b.truncated = dev_alloc<uint8_t>(P);
    b.counters = dev_alloc<uint64_t>(3 * slots);
    uint64_t *totals = dev_alloc<uint64_t>(3);

    check_hip(hipMemcpy(formation, form.data(), form.size() * sizeof(float), hipMemcpyHostToDevice),
              "hipMemcpy formation");
    // Env.__init__: native initial state (step index 0) and the fresh-env template
    check_rc(marlnav_formation_obs(&dims, formation, formation_obs, stream), "marlnav_formation_obs");
    check_rc(marlnav_reinit_all(&dims, &params, formation, b.states, b.obstacles, b.target, 0, stream),
             "marlnav_reinit_all");
    // the step loop: the policy's actions in, one launch per step (step k keys
    // the native re-init stream with k, as Env.step's k-th call does)
    for (int32_t k = 0; k < steps; ++k) {
        check_hip(hipMemcpyAsync(actions, acts.data() + (size_t)k * P * A * 2,
                                 (size_t)P * A * 2 * sizeof(float), hipMemcpyHostToDevice, stream),
                  "hipMemcpyAsync actions");
        check_rc(marlnav_step(&dims, &params, &b, (uint64_t)k + 1, stream), "marlnav_step");
    }
    check_rc(marlnav_counters_total(&dims, b.counters, totals, stream), "marlnav_counters_total");
    check_hip(hipStreamSynchronize(stream), "hipStreamSynchronize");

    std::FILE *out = std::fopen(argv[2], "wb");
    if (!out) die("cannot open output");
    put(out, b.states, P * A * 5);
    put(out, b.obstacles, P * S * 2);
    put(out, b.target, P * 2);
    put(out, b.step_num, P);
    put(out, b.terminates, P);
    put(out, b.obs, P * A * D);
    put(out, b.reward, P);
    put(out, b.terminated, P);
    put(out, b.truncated, P);
    put(out, totals, 3);
    std::fclose(out);
    std::printf("step_loop: %d steps of %lld envs x %d agents x %d obstacles\n", steps,
                (long long)P, A, O);
    return 0;
}
