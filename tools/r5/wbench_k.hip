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
    for (int K : {10, 20, 40, 60, 100}) {
        for (int mode = 0; mode < 3; ++mode) {
            // mode 0: the same K slots every launch; 1: consecutive launches walk the ring; 2: 4-wave blocks
            int k0 = 0;
            auto launch = [&]() {
                if (mode == 2)
                    hipLaunchKernelGGL((k_write<4>), dim3((unsigned)(B / 256)), dim3(256), 0, 0, obs, rew, done, B, P, K, k0, T);
                else
                    hipLaunchKernelGGL((k_write<1>), dim3((unsigned)(B / 64)), dim3(64), 0, 0, obs, rew, done, B, P, K, k0, T);
                if (mode == 1) k0 = (k0 + K) % T;
            };
            launch();
            CK(hipDeviceSynchronize());
            float best = 1e30f;
            for (int r = 0; r < 5; ++r) {
                CK(hipEventRecord(a));
                launch();
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                best = ms < best ? ms : best;
            }
            report(mode == 0 ? "same slots" : mode == 1 ? "ring walk" : "4-wave blocks", K, best, 1);
        }
        // back-to-back launches walking the ring, timed together
        {
            int k0 = 0;
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int r = 0; r < 5; ++r) {
                hipLaunchKernelGGL((k_write<1>), dim3((unsigned)(B / 64)), dim3(64), 0, 0, obs, rew, done, B, P, K, k0, T);
                k0 = (k0 + K) % T;
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            report("5 launches back to back, ring walk", K, ms, 5);
        }
    }
    return 0;
}
