// wbench.hip — the write roofline of the rollout's output pattern on MI355X.
//
// One lane per env, 64 envs per wave, K steps: per step every wave stores its 64 envs'
// obs block (64 x R x 32 B contiguous, 1 KB per store instruction, nontemporal), the
// rewards (64 x 4 B) and the done bytes (64 x 1 B) into ring slot k -- exactly what
// k_rollout_* write, with no env work.  Prints us per step for several shapes, next to a
// hipMemset fill of the same bytes.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/wbench tools/wbench.hip && /tmp/wbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <bool NT, bool SMALL, int LDSPAD = 0>
__global__ __launch_bounds__(256) void k_write(float4* obs, float* rew, unsigned char* done, long B, int P, int K,
                                               int work) {
    if constexpr (LDSPAD > 0) {  // occupancy limiter: LDSPAD bytes of LDS per block
        __shared__ int pad[LDSPAD / 4];
        if (threadIdx.x == 1023) pad[0] = 0;
    }
    const long env0 = (long)blockIdx.x * 256 + (threadIdx.x & ~63);
    const int lane = threadIdx.x & 63;
    const long slot = B * P;
    float acc = (float)lane;
    for (int k = 0; k < K; ++k) {
        for (int w = 0; w < work; ++w) acc = acc * 1.0001f + 0.5f;  // optional dependent VALU chain
        float4* ob = obs + k * slot + env0 * P;
        for (int it = 0; it < P; ++it) {
            float4 v = make_float4(acc, (float)it, (float)k, 1.f);
            if (NT) __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(ob + 64 * it + lane));
            else ob[64 * it + lane] = v;
        }
        if (SMALL) {
            rew[k * B + env0 + lane] = acc;
            done[k * B + env0 + lane] = (unsigned char)(k & 1);
        }
    }
}

// persistent grid: each wave takes 64-env chunks from an atomic counter (dynamic balance)
__global__ __launch_bounds__(256) void k_write_queue(float4* obs, float* rew, unsigned char* done, long B, int P, int K,
                                                     unsigned* counter) {
    const int lane = threadIdx.x & 63;
    const long slot = B * P;
    for (;;) {
        unsigned c = 0;
        if (lane == 0) c = atomicAdd(counter, 1u);
        c = __shfl(c, 0);
        const long env0 = (long)c * 64;
        if (env0 >= B) return;
        float acc = (float)lane;
        for (int k = 0; k < K; ++k) {
            float4* ob = obs + k * slot + env0 * P;
            for (int it = 0; it < P; ++it) {
                float4 v = make_float4(acc, (float)it, (float)k, 1.f);
                __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(ob + 64 * it + lane));
            }
            rew[k * B + env0 + lane] = acc;
            done[k * B + env0 + lane] = (unsigned char)(k & 1);
        }
    }
}

int main(int argc, char** argv) {
    const long B = 1 << 20;
    const int P = 18, T = 100;
    float4* obs;
    float* rew;
    unsigned char* done;
    CK(hipMalloc(&obs, (size_t)T * B * P * 16));
    CK(hipMalloc(&rew, (size_t)T * B * 4));
    CK(hipMalloc(&done, (size_t)T * B));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = (int)(B / 256);
    auto run = [&](const char* name, auto launch, int K) {
        if (K > 3 * T) { printf("K too large\n"); exit(1); }
        launch(K);
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(a));
            launch(K);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        const double us = best * 1e3 / K;
        const double bytes = (double)B * (P * 16 + 5);
        printf("{\"shape\": \"%s\", \"K\": %d, \"us_per_step\": %.2f, \"TB_s\": %.3f}\n", name, K, us, bytes / us / 1e6);
    };
    unsigned* counter;
    CK(hipMalloc(&counter, 4));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int K : {20, 100}) {
        run("nt, 4 waves/SIMD (LDS-limited)", [&](int k) { hipLaunchKernelGGL((k_write<true, true, 40960>), dim3(grid), dim3(256), 0, 0, obs, rew, done, B, P, k, 0); }, K);
        run("nt, 2 waves/SIMD (LDS-limited)", [&](int k) { hipLaunchKernelGGL((k_write<true, true, 81920>), dim3(grid), dim3(256), 0, 0, obs, rew, done, B, P, k, 0); }, K);
        run("nt, atomic queue 4 blocks/CU", [&](int k) {
            CK(hipMemsetAsync(counter, 0, 4));
            hipLaunchKernelGGL(k_write_queue, dim3(cus * 4), dim3(256), 0, 0, obs, rew, done, B, P, k, counter); }, K);
        // (k <= T: every launch writes ring slots 0 .. k - 1)
        run("3 back-to-back launches", [&](int k) {
            for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_write<true, true>), dim3(grid), dim3(256), 0, 0, obs, rew, done, B, P, k / 3, 0); }, 3 * K);
        run("nt obs+rew+done", [&](int k) { hipLaunchKernelGGL((k_write<true, true>), dim3(grid), dim3(256), 0, 0, obs, rew, done, B, P, k, 0); }, K);
        run("nt obs only", [&](int k) { hipLaunchKernelGGL((k_write<true, false>), dim3(grid), dim3(256), 0, 0, obs, rew, done, B, P, k, 0); }, K);
        run("plain obs+rew+done", [&](int k) { hipLaunchKernelGGL((k_write<false, true>), dim3(grid), dim3(256), 0, 0, obs, rew, done, B, P, k, 0); }, K);
        run("nt + 400 VALU/step", [&](int k) { hipLaunchKernelGGL((k_write<true, true>), dim3(grid), dim3(256), 0, 0, obs, rew, done, B, P, k, 400); }, K);
        run("memset same bytes", [&](int k) {
            CK(hipMemsetAsync(obs, 0, (size_t)k * B * P * 16));
            CK(hipMemsetAsync(rew, 0, (size_t)k * B * 4));
            CK(hipMemsetAsync(done, 0, (size_t)k * B));
        }, K);
    }
    return 0;
}
