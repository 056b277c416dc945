// wbench_sizes.hip — the write floor of k_rollout_lean's output pattern at the strong-scaling
// shard sizes (131,072 / 262,144 / 2^20 envs, R = 9, K = 20 / 100): what a kernel that only
// stores the obs / reward / done stream (no env work) achieves, next to hipMemset of the same
// bytes and an empty launch of the same grid.
//   hipcc -O3 --offload-arch=gfx950 -o exp/wbench_sizes tools/r5/wbench_sizes.hip && exp/wbench_sizes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                              \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

// one 64-env group per 64-thread block (k_rollout_lean's grid); LDSB bytes of LDS per block
// limit the waves per CU as the real kernel's image does (10 KB: 16 per CU)
template <int LDSB, int GROUPS, int ROT = 0>
__global__ __launch_bounds__(64) void k_write(float4* obs, float* rew, unsigned char* done, long B, int P, int K,
                                              long ngroups) {
    __shared__ int pad[LDSB / 4];
    if (threadIdx.x == 1023) pad[0] = 0;
    const int lane = threadIdx.x;
    const long slot = B * P;
    float acc = (float)lane;
    for (int k = 0; k < K; ++k) {
        for (int g = 0; g < GROUPS; ++g) {  // GROUPS > 1: persistent waves, groups strided by the grid
            const long grp = (long)blockIdx.x + (long)g * gridDim.x;
            if (grp >= ngroups) break;
            const long env0 = grp * 64;
            float4* ob = obs + k * slot + env0 * P;
            // ROT: the wave issues its P store instructions starting from a per-wave offset, so
            // waves in lockstep write different 1-KB pieces of their blocks at the same time
            const int r0 = ROT == 1 ? (int)(grp % P) : ROT == 2 ? (int)((grp * 7) % P) : 0;
            for (int j = 0; j < P; ++j) {
                int it = j + r0;
                if (it >= P) it -= P;
                if (ROT == 3 && (grp & 1)) it = P - 1 - j;
                float4 v = make_float4(acc, (float)it, (float)k, 1.f);
                __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(ob + 64 * it + lane));
            }
            __builtin_nontemporal_store(acc, rew + k * B + env0 + lane);
            __builtin_nontemporal_store((unsigned char)(k & 1), done + k * B + env0 + lane);
        }
    }
}
__global__ void k_empty(int* x) {
    if (threadIdx.x == 1023) x[0] = 0;
}

int main() {
    const int P = 18, T = 100;
    const long BMAX = 1 << 20;
    float4* obs;
    float* rew;
    unsigned char* done;
    int* dummy;
    CK(hipMalloc(&obs, (size_t)T * BMAX * P * 16));
    CK(hipMalloc(&rew, (size_t)T * BMAX * 4));
    CK(hipMalloc(&done, (size_t)T * BMAX));
    CK(hipMalloc(&dummy, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (long B : {131072L, 262144L, 1048576L}) {
        const long ng = B / 64;
        auto run = [&](const char* name, auto launch, int K) {
            launch(K);
            CK(hipDeviceSynchronize());
            float best = 1e30f, sum = 0;
            for (int r = 0; r < 5; ++r) {
                CK(hipEventRecord(a));
                launch(K);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                best = ms < best ? ms : best;
                sum += ms;
            }
            const double us = best * 1e3 / (K > 0 ? K : 1);
            const double bytes = (double)B * (P * 16 + 5);
            printf("{\"envs\": %ld, \"shape\": \"%s\", \"K\": %d, \"us_per_step\": %.3f, \"mean_us_per_step\": %.3f, \"TB_s\": %.3f}\n",
                   B, name, K, us, sum * 1e3 / 5 / (K > 0 ? K : 1), K > 0 ? bytes / us / 1e6 : 0.0);
        };
        for (int K : {20, 100}) {
            run("lean grid, 10 KB LDS (4 waves/SIMD)", [&](int k) {
                hipLaunchKernelGGL((k_write<10240, 1>), dim3((unsigned)ng), dim3(64), 0, 0, obs, rew, done, B, P, k, ng); }, K);
            run("lean grid, 10 KB LDS, store order rotated by wave", [&](int k) {
                hipLaunchKernelGGL((k_write<10240, 1, 1>), dim3((unsigned)ng), dim3(64), 0, 0, obs, rew, done, B, P, k, ng); }, K);
            run("lean grid, 10 KB LDS, store order rotated by 7 x wave", [&](int k) {
                hipLaunchKernelGGL((k_write<10240, 1, 2>), dim3((unsigned)ng), dim3(64), 0, 0, obs, rew, done, B, P, k, ng); }, K);
            run("lean grid, 10 KB LDS, odd waves reversed", [&](int k) {
                hipLaunchKernelGGL((k_write<10240, 1, 3>), dim3((unsigned)ng), dim3(64), 0, 0, obs, rew, done, B, P, k, ng); }, K);
            run("lean grid, 20 KB LDS (2 waves/SIMD)", [&](int k) {
                hipLaunchKernelGGL((k_write<20480, 1>), dim3((unsigned)ng), dim3(64), 0, 0, obs, rew, done, B, P, k, ng); }, K);
            run("lean grid, 4 KB LDS (8 waves/SIMD)", [&](int k) {
                hipLaunchKernelGGL((k_write<4096, 1>), dim3((unsigned)ng), dim3(64), 0, 0, obs, rew, done, B, P, k, ng); }, K);
            if (ng > 4096) run("persistent 4096 waves, groups looped per step", [&](int k) {
                hipLaunchKernelGGL((k_write<10240, 4>), dim3(4096), dim3(64), 0, 0, obs, rew, done, B, P, k, ng); }, K);
            run("memset same bytes", [&](int k) {
                CK(hipMemsetAsync(obs, 0, (size_t)k * B * P * 16));
                CK(hipMemsetAsync(rew, 0, (size_t)k * B * 4));
                CK(hipMemsetAsync(done, 0, (size_t)k * B));
            }, K);
        }
        run("empty launch, lean grid", [&](int k) {
            hipLaunchKernelGGL(k_empty, dim3((unsigned)ng), dim3(64), 0, 0, dummy); }, 0);
    }
    return 0;
}
