// wbench_k.hip — the store-only stream of k_rollout_lean's outputs at 2^20 envs (R = 9), by launch
// length and placement: why a 20-step launch writes at 5.7 TB/s and a 100-step one at 6.8.
//   hipcc -O3 --offload-arch=gfx950 -o exp/wbench_k tools/r5/wbench_k.hip && exp/wbench_k
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                              \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

// one 64-env group per wave, NW waves per block; steps k0 .. k0 + K - 1 of a T-slot ring
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_write(float4* obs, float* rew, unsigned char* done, long B, int P, int K,
                                                   int k0, int T) {
    __shared__ int pad[2560 * NW];
    if (threadIdx.x == 100000) pad[0] = 0;
    const int lane = threadIdx.x & 63;
    const long grp = (long)blockIdx.x * NW + (threadIdx.x >> 6);
    const long env0 = grp * 64;
    if (env0 >= B) return;
    float acc = (float)lane;
    for (int k = 0; k < K; ++k) {
        const long s = (k0 + k) % T;
        float4* ob = obs + s * B * P + env0 * P;
        for (int j = 0; j < P; ++j) {
            float4 v = make_float4(acc, (float)j, (float)k, 1.f);
            __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(ob + 64 * j + lane));
        }
        __builtin_nontemporal_store(acc, rew + s * B + env0 + lane);
        __builtin_nontemporal_store((unsigned char)(k & 1), done + s * B + env0 + lane);
    }
}

int main() {
    const int P = 18, T = 100;
    const long B = 1L << 20;
    float4* obs;
    float* rew;
    unsigned char* done;
    CK(hipMalloc(&obs, (size_t)T * B * P * 16));
    CK(hipMalloc(&rew, (size_t)T * B * 4));
    CK(hipMalloc(&done, (size_t)T * B));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double bytes = (double)B * (P * 16 + 5);
    auto report = [&](const char* name, int K, float ms, int launches) {
        const double us = ms * 1e3 / ((double)K * launches);
        printf("{\"shape\": \"%s\", \"K\": %d, \"launches\": %d, \"us_per_step\": %.3f, \"TB_s\": %.3f}\n", name, K,
               launches, us, bytes / us / 1e6);
        fflush(stdout);
    };
    // K = 20 by where the timed launch writes: the slots the previous launch wrote ("same"),
    // slots last written 2 / 5 launches before (a 40 / 100-slot ring), or never-written memory
    // (a 48 GB region walked once)
    {
        const int K = 20;
        const long FRESH_SLOTS = 160;  // 48 GB of obs at 2^20 envs
        float4* big;
        CK(hipMalloc(&big, (size_t)FRESH_SLOTS * B * P * 16));
        for (int rep = 0; rep < 2; ++rep) {
            for (int mode = 0; mode < 4; ++mode) {
                const int TT = mode == 0 ? K : mode == 1 ? 2 * K : 100;
                int k0 = 0;
                long fresh = 0;
                auto launch = [&]() {
                    if (mode == 3) {
                        hipLaunchKernelGGL((k_write<1>), dim3((unsigned)(B / 64)), dim3(64), 0, 0, big + fresh * B * P, rew,
                                           done, B, P, K, 0, T);
                        fresh += K;
                    } else {
                        hipLaunchKernelGGL((k_write<1>), dim3((unsigned)(B / 64)), dim3(64), 0, 0, obs, rew, done, B, P, K,
                                           k0, TT);
                        k0 = (k0 + K) % TT;
                    }
                };
                for (int w = 0; w < 5; ++w) launch();  // (fresh: the first 100 slots written)
                CK(hipDeviceSynchronize());
                float best = 1e30f, sum = 0.f;
                for (int r = 0; r < 3; ++r) {
                    CK(hipEventRecord(a));
                    launch();
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    float ms;
                    CK(hipEventElapsedTime(&ms, a, b));
                    best = ms < best ? ms : best;
                    sum += ms;
                }
                report(mode == 0 ? "K=20: the slots of the previous launch" : mode == 1 ? "K=20: slots written 2 launches before"
                       : mode == 2 ? "K=20: slots written 5 launches before" : "K=20: never-written memory", K, best, 1);
                report(mode == 0 ? "  mean of 3" : mode == 1 ? "  mean of 3" : mode == 2 ? "  mean of 3" : "  mean of 3", K,
                       sum / 3, 1);
            }
        }
        CK(hipFree(big));
    }
    return 0;
}
