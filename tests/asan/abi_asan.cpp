// Host-side AddressSanitizer / UBSan driver for the C ABI of liblbk8s (include/lbk8s.h).
// SURVEY §5 "Race detection / sanitizers": the kernels run per env with no cross-env
// state, so the sanitizable surface is the host code of the entry points — config
// validation, state-blob layout arithmetic, argument checks, error reporting and the
// launch paths' host side.  Built with the device code unsanitized
// (-Xarch_host -fsanitize=address,undefined) and run without a GPU: every launch must fail
// cleanly (an error code and a message), never crash or touch memory it does not own.
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "lbk8s.h"

static int failures = 0;
#define CHECK(cond)                                                          \
    do {                                                                     \
        if (!(cond)) {                                                       \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                      \
        }                                                                    \
    } while (0)

static lb_config base_cfg() {
    lb_config c;
    std::memset(&c, 0, sizeof(c));
    c.num_endpoints = 8; c.num_zones = 4; c.num_nodes = 24; c.episode_length = 100;
    c.reward_fn = LB_REWARD_NAIVE; c.rejection_allowed = 1; c.auto_reset = 1; c.rng_mode = LB_RNG_PHILOX;
    c.arrival_rate = 100.0; c.call_duration = 1.0; c.latency_weight = 0.7; c.cpu_weight = 0.1; c.gini_weight = 0.2;
    return c;
}

int main() {
    CHECK(lb_abi_version() == LBK8S_ABI_VERSION);
    lb_config c = base_cfg();
    CHECK(lb_validate_config(&c) == 0);
    CHECK(lb_validate_config(nullptr) != 0);
    // every constructor constraint of the reference (and the ABI's own limits)
    struct { int field; int value; const char* word; } bad[] = {
        {0, 0, "num_endpoints"}, {0, 257, "num_endpoints"}, {1, 3, "IndexError"}, {2, 23, "IndexError"},
        {2, 257, "num_nodes"}, {3, 0, "episode_length"}, {3, 1024, "episode_length"}, {4, 4, "reward"},
        {5, 0, nullptr}, {6, 0, nullptr}, {7, 2, "rng_mode"}, {8, 3, "geometry"}};
    for (auto& b : bad) {
        lb_config x = base_cfg();
        int* f[] = {&x.num_endpoints, &x.num_nodes, &x.num_nodes, &x.episode_length, &x.reward_fn,
                    &x.rejection_allowed, &x.auto_reset, &x.rng_mode, &x.geometry};
        if (b.field == 1) x.num_zones = b.value; else *f[b.field] = b.value;
        const int rc = lb_validate_config(&x);
        if (b.word) {
            CHECK(rc != 0);
            CHECK(std::strstr(lb_last_error(), b.word) != nullptr);
        } else {
            CHECK(rc == 0);  // rejection off / auto-reset off are valid
        }
    }
    {
        lb_config x = base_cfg();
        x.arrival_rate = 0.0;
        CHECK(lb_validate_config(&x) != 0);
    }
    // state layout: every (geometry, E, B) combination, including B past 2^32 bytes of state
    uint64_t prev = 0;
    for (int g = 0; g <= 2; ++g)
        for (int E : {1, 3, 6, 8, 9, 16, 17, 64, 100, 256})
            for (int64_t B : {1LL, 63LL, 64LL, 4096LL, 32767LL, 32768LL, 262144LL, 1LL << 20, 1LL << 26}) {
                lb_config x = base_cfg();
                x.num_endpoints = E;
                x.geometry = g;
                uint64_t n = 0;
                CHECK(lb_state_bytes(&x, B, &n) == 0);
                CHECK(n % 256 == 0 && n > (uint64_t)B * 8);
                if (E == 8 && g == 0 && B == 4096) prev = n;
            }
    CHECK(prev > 0);
    uint64_t n = 0;
    CHECK(lb_state_bytes(&c, 0, &n) != 0);
    CHECK(lb_state_bytes(&c, 16, nullptr) != 0);
    // argument checks of every entry point (no device memory is touched: NULL / bad args)
    CHECK(lb_init(nullptr, &c, 16, nullptr, nullptr) != 0);
    CHECK(lb_reset(nullptr, &c, 16, nullptr, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_step(nullptr, &c, 16, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_rollout(nullptr, &c, 16, 0, 4, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_policy(nullptr, &c, 16, 0, nullptr, nullptr) != 0);
    CHECK(lb_get_field(nullptr, &c, 16, 0, nullptr, nullptr) != 0);
    CHECK(lb_get_stats(nullptr, &c, 16, nullptr, nullptr) != 0);
    CHECK(lb_status(nullptr, &c, 16, nullptr, nullptr) != 0);
    CHECK(lb_ds_pack(nullptr, nullptr, nullptr) != 0);
    CHECK(lb_ds_forward(nullptr, nullptr, 1, 9, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_ds_q_argmax(nullptr, nullptr, 1, 9, nullptr, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_ds_train_forward(nullptr, nullptr, 1, 9, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_ds_pack_backward(nullptr, nullptr, nullptr) != 0);
    CHECK(lb_ds_train_backward(nullptr, nullptr, 1, 9, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                               nullptr) != 0);
    CHECK(lb_ppo_head(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 1, 9, 0.2f, 0.f, 0.5f, 1,
                      nullptr, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_replay_add(1, 72, 4, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                        nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_dqn_act(nullptr, nullptr, 16, 9, nullptr, nullptr, &c, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_dqn_head(nullptr, nullptr, nullptr, nullptr, nullptr, 1, 9, 0.99f, nullptr, nullptr, nullptr, nullptr,
                      nullptr, nullptr) != 0);
    CHECK(lb_ds_pack_pair(nullptr, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_ds_forward_pair(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 1, 9, nullptr) != 0);
    CHECK(lb_dqn_steps(nullptr, nullptr, 16, 9, nullptr, nullptr, &c, nullptr, nullptr, nullptr, nullptr, nullptr,
                       nullptr, nullptr, 4, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                       nullptr, 0, nullptr, nullptr) != 0);
    CHECK(lb_replay_sample(1, 72, 4, 8, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                           nullptr, nullptr, nullptr, nullptr, nullptr) != 0);
    CHECK(lb_ds_set_grads(nullptr, nullptr, nullptr, 1, 9, nullptr, nullptr) != 0);
    // out-of-range arguments past the NULL checks (fake, never-dereferenced pointers)
    void* fake = reinterpret_cast<void*>(0x1000);
    CHECK(lb_ds_set_grads((const float*)fake, (const float*)fake, nullptr, 1, LB_DS_MAX_ELEMENTS_TRAIN + 1,
                          (float*)fake, nullptr) != 0);
    CHECK(lb_ds_set_grads((const float*)fake, (const float*)fake, nullptr, 0, 9, (float*)fake, nullptr) != 0);
    {  // head loss_out above one block, paired forward past 16 elements
        float* ff = (float*)fake;
        CHECK(lb_dqn_head(ff, ff, (const int64_t*)fake, ff, ff, 2000, 9, 0.99f, ff, ff, nullptr, nullptr, ff, nullptr) != 0);
        CHECK(lb_ds_forward_pair(ff, ff, ff, ff, ff, ff, ff, ff, 128, 17, nullptr) != 0);
    }
    CHECK(lb_policy(fake, &c, 16, 9, (int32_t*)fake, nullptr) != 0);
    CHECK(lb_get_field(fake, &c, 16, LB_FIELD_COUNT, (double*)fake, nullptr) != 0);
    CHECK(lb_get_field(fake, &c, 16, LB_FIELD_DT, (double*)fake, nullptr) != 0);
    CHECK(lb_ds_forward((const float*)fake, (const float*)fake, 1, 0, (float*)fake, nullptr, nullptr) != 0);
    CHECK(lb_ds_forward((const float*)fake, (const float*)fake, 1, LB_DS_MAX_ELEMENTS_FWD + 1, (float*)fake, nullptr,
                        nullptr) != 0);
    CHECK(lb_ds_train_forward((const float*)fake, (const float*)fake, 1, LB_DS_MAX_ELEMENTS_TRAIN + 1, (float*)fake,
                              nullptr, (float*)fake, nullptr, (float*)fake, nullptr) != 0);
    {
        lb_config t = base_cfg();
        t.rng_mode = LB_RNG_TRACE;
        CHECK(lb_step(fake, &t, 16, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) != 0);
        CHECK(lb_rollout(fake, &t, 16, 3, 4, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) != 0);
        lb_trace tr;
        std::memset(&tr, 0, sizeof(tr));
        CHECK(lb_init(fake, &t, 16, &tr, nullptr) != 0);  // trace mode needs t0
        CHECK(std::strstr(lb_last_error(), "t0") != nullptr);
    }
    // the launch paths' host side without a GPU: a clean error, never a crash
    {
        const int rc = lb_policy(fake, &c, 16, LB_POLICY_RANDOM, (int32_t*)fake, nullptr);
        CHECK(rc == 0 || std::strlen(lb_last_error()) > 0);
    }
    // lb_last_error is thread-local
    lb_validate_config(nullptr);
    std::vector<std::thread> th;
    std::vector<int> ok(4, 0);
    for (int i = 0; i < 4; ++i)
        th.emplace_back([i, &ok] {
            lb_config x = base_cfg();
            x.num_nodes = 10;
            lb_validate_config(&x);
            ok[i] = std::strstr(lb_last_error(), "IndexError") != nullptr;
        });
    for (auto& t : th) t.join();
    for (int v : ok) CHECK(v);
    CHECK(std::strstr(lb_last_error(), "NULL") != nullptr);
    std::printf("abi_asan: %s (%d failures)\n", failures ? "FAIL" : "ok", failures);
    return failures ? 1 : 0;
}
