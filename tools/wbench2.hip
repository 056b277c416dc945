// wbench2.hip -- where the rollout's fixed launch cost comes from, on the store pattern alone.
//
// The k_rollout_img output stream (2^20 envs, R = 9: per step every wave stores its 64 envs'
// obs block, 64 x 288 B contiguous, as 18 nontemporal 1 KB store instructions, plus the
// rewards and done bytes into ring slot k) written by different grid shapes, K = 20 and 100:
//   gen4      one 64-env group per wave, 4096 blocks of 256 (40 KB LDS each: 4 blocks per CU,
//             the rollout's occupancy) -> four block generations (tools/wbench.hip's shape)
//   static4   exactly the resident grid (4 blocks per CU), each wave runs its four groups one
//             after the other (group g = wave + i * waves): no block dispatch after the start
//   inter4    the resident grid, each wave interleaves its four groups step by step (k outer):
//             every wave is at the same step for the whole launch
//   gen4+ld   gen4 plus one dependent 8-byte table load per step issued AFTER the step's stores
//             (vmcnt is in order: its use waits for every older store of the wave)
//   gen4+ldF  the same load issued BEFORE the step's stores, used after them
//   memset    hipMemsetAsync of the same bytes
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/wbench2 tools/wbench2.hip && /tmp/wbench2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                            \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int P = 18;

__device__ __forceinline__ void pad_lds() {
    __shared__ int pad[40960 / 4];
    if (threadIdx.x == 1023) pad[0] = 0;  // never true: only reserves the LDS
}

__device__ __forceinline__ void store_step(float4* obs, float* rew, unsigned char* done, long B, long env0, int lane,
                                           int k, float acc) {
    float4* ob = obs + (long)k * B * P + env0 * P;
#pragma unroll
    for (int it = 0; it < P; ++it)
        __builtin_nontemporal_store(f4v{acc, (float)it, (float)k, 1.f}, reinterpret_cast<f4v*>(ob + 64 * it + lane));
    __builtin_nontemporal_store(acc, rew + (long)k * B + env0 + lane);
    __builtin_nontemporal_store((unsigned char)(k & 1), done + (long)k * B + env0 + lane);
}

// LD: 0 none, 1 load after the stores (used at the next step), 2 load before the stores
template <int LD>
__global__ __launch_bounds__(256) void k_gen(float4* obs, float* rew, unsigned char* done, long B, int K,
                                             const double* tab) {
    pad_lds();
    const long env0 = (long)blockIdx.x * 256 + (threadIdx.x & ~63);
    const int lane = threadIdx.x & 63;
    float acc = (float)lane;
    unsigned idx = (unsigned)(env0 + lane) & 4095u;
    double v = 0.0;
    for (int k = 0; k < K; ++k) {
        if (LD == 2) v = tab[idx];
        store_step(obs, rew, done, B, env0, lane, k, acc);
        if (LD == 2) { acc += (float)v; idx = (idx * 1664525u + (unsigned)v) & 4095u; }
        if (LD == 1) { acc += (float)v; v = tab[idx]; idx = (idx * 1664525u + (unsigned)k) & 4095u; }
    }
    if (acc == -1.f) rew[0] = acc;
}

template <bool INTER>
__global__ __launch_bounds__(256) void k_static(float4* obs, float* rew, unsigned char* done, long B, int K, int G) {
    pad_lds();
    const long nw = (long)gridDim.x * 4;
    const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    float acc = (float)lane;
    if (INTER) {
        for (int k = 0; k < K; ++k)
            for (int g = 0; g < G; ++g) {
                const long env0 = (w + g * nw) * 64;
                if (env0 < B) store_step(obs, rew, done, B, env0, lane, k, acc);
            }
    } else {
        for (int g = 0; g < G; ++g) {
            const long env0 = (w + g * nw) * 64;
            if (env0 >= B) break;
            for (int k = 0; k < K; ++k) store_step(obs, rew, done, B, env0, lane, k, acc);
        }
    }
}

int main(int argc, char** argv) {
    const long B = 1 << 20;
    const int T = 100;
    float4* obs;
    float* rew;
    unsigned char* done;
    double* tab;
    CK(hipMalloc(&obs, (size_t)T * B * P * 16));
    CK(hipMalloc(&rew, (size_t)T * B * 4));
    CK(hipMalloc(&done, (size_t)T * B));
    CK(hipMalloc(&tab, 4096 * 8));
    CK(hipMemset(tab, 0, 4096 * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = (int)(B / 256), sgrid = cus * 4;
    const int G = (int)((B / 64 + sgrid * 4 - 1) / (sgrid * 4));
    auto run = [&](const char* name, auto launch, int K) {
        launch(K);
        CK(hipDeviceSynchronize());
        float best = 1e30f, sum = 0.f;
        const int reps = 5;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(a));
            launch(K);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
            sum += ms;
        }
        const double us = best * 1e3 / K;
        const double bytes = (double)B * (P * 16 + 5);
        printf("{\"shape\": \"%s\", \"K\": %d, \"us_per_step_best\": %.2f, \"us_per_step_mean\": %.2f, \"TB_s\": %.3f}\n",
               name, K, us, sum / reps * 1e3 / K, bytes / us / 1e6);
        fflush(stdout);
    };
    for (int K : {20, 100}) {
        run("gen4", [&](int k) { hipLaunchKernelGGL(k_gen<0>, dim3(grid), dim3(256), 0, 0, obs, rew, done, B, k, tab); }, K);
        run("static4", [&](int k) { hipLaunchKernelGGL(k_static<false>, dim3(sgrid), dim3(256), 0, 0, obs, rew, done, B, k, G); }, K);
        run("inter4", [&](int k) { hipLaunchKernelGGL(k_static<true>, dim3(sgrid), dim3(256), 0, 0, obs, rew, done, B, k, G); }, K);
        run("gen4+ld", [&](int k) { hipLaunchKernelGGL(k_gen<1>, dim3(grid), dim3(256), 0, 0, obs, rew, done, B, k, tab); }, K);
        run("gen4+ldF", [&](int k) { hipLaunchKernelGGL(k_gen<2>, dim3(grid), dim3(256), 0, 0, obs, rew, done, B, k, tab); }, K);
        run("memset", [&](int k) {
            CK(hipMemsetAsync(obs, 0, (size_t)k * B * P * 16));
            CK(hipMemsetAsync(rew, 0, (size_t)k * B * 4));
            CK(hipMemsetAsync(done, 0, (size_t)k * B));
        }, K);
    }
    return 0;
}
