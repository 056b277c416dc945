// lbk8s.hip — MI355X (gfx950) kernels + C ABI for the vectorized LoadBalancerK8sEnv.
//
// Reference hot path: /root/reference/envs/loadbalancer_k8s_env.py (reset :290-400,
// step :403-513, take_action :578-686, get_reward :516-567, get_state :688-758,
// next_request :1131-1163), envs/utils.py (gini :132-143, endpoint list :33-64) and
// envs/baselines.py (greedy policies :6-35).  Public ABI: include/lbk8s.h; design
// notes: DESIGN.md.
//
// Two state layouts / kernel shapes share one state representation (lbk8s_common.h):
//   * E <= 8 : k_step_tpe    — one lane per env, LDS-staged coalesced obs (lbk8s_tpe.h);
//              k_rollout_tpe — K steps per launch, the env in registers (lb_rollout)
//   * E >  8 : k_step_slice  — one W-lane slice per env (4 envs per wave up to E = 64),
//                              lanes over endpoints; k_rollout_slice (lbk8s_slice.h)

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>

#include "lbk8s.h"
#include "lbk8s_common.h"
#include "lbk8s_deepsets.h"
#include "lbk8s_ds_train.h"
#include "lbk8s_dqn.h"
#include "lbk8s_slice.h"
#include "lbk8s_tpe.h"
#include "lbk8s_rollout.h"
#include "lbk8s_lean_launch.h"

namespace lbk {

// lb_replay_add: the DQN vector step's bookkeeping in one launch (dqn_deepset.py:158-174
// replay add + obs <- next_obs, :147-156 episode returns).  Slot pos = *pos_in; one thread
// writes (pos + 1) % slots to *pos_out, a different word (callers alternate the two), so
// no thread of this launch can read the advanced position.
struct ReplayParams {
    int64_t B;
    int f4;  // float4s per observation
    int64_t slots;
    const int64_t* pos_in;
    int64_t* pos_out;
    float4* obs;
    const float4* next_obs;
    const int32_t* actions;
    const float* reward;
    const uint8_t* done;
    const double* ep_stats;  // [B][LB_ST_K], column 0 = the finished episode's return
    float4* rb_obs;
    float4* rb_next_obs;
    int64_t* rb_actions;
    float* rb_rewards;
    float* rb_dones;
    double* ep_sum;  // [B] per-env sums (deterministic; reduced when flushed)
    double* ep_cnt;
};

__global__ void k_replay_add(ReplayParams p) {
    const int64_t pos = *p.pos_in;
    const int64_t n4 = p.B * p.f4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4 || i < p.B;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (i < n4) {
            const float4 o = p.obs[i], nx = p.next_obs[i];
            p.rb_obs[pos * n4 + i] = o;
            p.rb_next_obs[pos * n4 + i] = nx;
            p.obs[i] = nx;
        }
        if (i < p.B) {
            const float d = p.done[i] ? 1.f : 0.f;
            p.rb_actions[pos * p.B + i] = p.actions[i];
            p.rb_rewards[pos * p.B + i] = p.reward[i];
            p.rb_dones[pos * p.B + i] = d;
            if (p.ep_sum && p.done[i]) {
                p.ep_sum[i] += p.ep_stats[i * LB_ST_K];
                p.ep_cnt[i] += 1.0;
            }
        }
        if (i == 0) *p.pos_out = (pos + 1) % p.slots;
    }
}

// lb_replay_sample: SB3 ReplayBuffer.sample's (slot, env) draws and the gather; thread
// (i, part): part < f4 -> obs float4, < 2 f4 -> next_obs float4, == 2 f4 -> the scalars
struct ReplaySampleParams {
    int64_t B;
    int f4;
    int64_t slots;
    int batch;
    uint64_t seed;
    const int64_t* vstep;
    const int64_t* base_adds;
    const float4* rb_obs;
    const float4* rb_next_obs;
    const int64_t* rb_actions;
    const float* rb_rewards;
    const float* rb_dones;
    float4* obs;
    float4* next_obs;
    int64_t* actions;
    float* rewards;
    float* dones;
};
__global__ void k_replay_sample(ReplaySampleParams p) {
    const int parts = 2 * p.f4 + 1;
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (int64_t)p.batch * parts) return;
    const int i = (int)(q / parts), part = (int)(q - (int64_t)i * parts);
    const int64_t t = *p.vstep, adds = *p.base_adds + t;
    const int64_t upper = adds < p.slots ? (adds > 0 ? adds : 1) : p.slots;
    const U4 w = philox((uint32_t)t, (uint32_t)((uint64_t)t >> 32), (uint32_t)i, D_DQN_SAMPLE, (uint32_t)p.seed,
                        (uint32_t)(p.seed >> 32));
    const int64_t bi = (int64_t)(((uint64_t)w.x * (uint64_t)upper) >> 32);  // upper < 2^32
    const int64_t ei = (int64_t)bounded(w.y, (uint32_t)p.B);
    const int64_t row = bi * p.B + ei;
    if (part < p.f4) p.obs[(int64_t)i * p.f4 + part] = p.rb_obs[row * p.f4 + part];
    else if (part < 2 * p.f4) p.next_obs[(int64_t)i * p.f4 + part - p.f4] = p.rb_next_obs[row * p.f4 + part - p.f4];
    else {
        p.actions[i] = p.rb_actions[row];
        p.rewards[i] = p.rb_rewards[row];
        p.dones[i] = p.rb_dones[row];
    }
}

// lb_episode_log: VecMonitor's per-env float32 return and the finished episodes' rows,
// appended to a device log (one atomic per wave: the ballot's count)
struct EpLogParams {
    int64_t B;
    const uint8_t* done;
    const double* ep_stats;
    const float* reward;
    const double* reward64;
    const int32_t* actions;
    float* ret32;
    float* ep_r32;
    int64_t tag;
    double* log;
    int64_t cap;
    uint32_t* count;
};

__global__ __launch_bounds__(256) void k_episode_log(EpLogParams p) {
    const int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool live = env < p.B;
    bool d = false;
    float r32 = 0.f;
    if (live) {
        // VecMonitor's float32 episode_returns += the env's float64 reward: one rounding
        r32 = p.reward64 ? (float)((double)p.ret32[env] + p.reward64[env]) : p.ret32[env] + p.reward[env];
        d = p.done[env] != 0;
        p.ret32[env] = d ? 0.f : r32;
        if (d && p.ep_r32) p.ep_r32[env] = r32;
    }
    const uint64_t m = __ballot(d);
    if (!m) return;
    uint32_t base = 0;
    if (lane == __ffsll((unsigned long long)m) - 1) base = atomicAdd(p.count, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, __ffsll((unsigned long long)m) - 1);
    if (!d) return;
    const int64_t slot = (int64_t)base + __popcll(m & ((1ull << lane) - 1));
    if (slot >= p.cap) return;
    double* row = p.log + slot * LB_EPLOG_W;
    const double* st = p.ep_stats + env * LB_ST_K;
#pragma unroll
    for (int k = 0; k < LB_ST_K; ++k) row[k] = st[k];
    row[LB_EPLOG_RET32] = (double)r32;
    row[LB_EPLOG_REWARD] = (double)p.reward[env];
    row[LB_EPLOG_ACTION] = (double)p.actions[env];
    row[LB_EPLOG_ENV] = (double)env;
    row[LB_EPLOG_TAG] = (double)p.tag;
}

// LAT[k][j]: endpoint latency after j selections from trunc(initial) = k
// (increase_endpoint_latency :1013-1023 then decrease_endpoint_latency :1052-1060 in the
// same step); CPU[c][M]: node cpu after M selections (:861-887 then :937-960).
__global__ void k_luts(double* lat_lut, double* cpu_lut) {
    int row = blockIdx.x * blockDim.x + threadIdx.x;
    // column-major ([j][k]): envs stepping in lockstep hold similar counters, so one
    // step's lookups touch a few columns (L1/L2-resident) rather than scattered rows
    if (row < LAT_ROWS) {
        double v = (double)row;
        lat_lut[row] = v;
        for (int j = 1; j < JCAP; ++j) {
            double inc = clamp_lat(trunc(v) * 1.5);
            v = clamp_lat(trunc(inc) / 1.15);
            lat_lut[(int64_t)j * LAT_ROWS + row] = v;
        }
    } else if (row < LAT_ROWS + CPU_ROWS) {
        int c = row - LAT_ROWS;
        double w = (double)c;
        cpu_lut[c] = w;
        for (int m = 1; m < JCAP; ++m) {
            w = clamp_cpu(clamp_cpu(w * 1.15) / 1.15);
            cpu_lut[(int64_t)m * CPU_ROWS + c] = w;
        }
    }
}

// __init__ (:86-287): the only state that reaches reset() is current_time, advanced by
// __init__'s own next_request() (:267).
__global__ void k_init(Params p, int trace) {
    int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= p.B) return;
    for (int e = 0; e < p.EP; ++e) {
        int64_t i = eidx(p, env, e);
        p.lat0[i] = 0.0;
        p.emeta[i] = 0;
        p.edyn[i] = 0;
    }
    double t;
    if (trace) {
        t = p.tr.t0[env];
    } else {
        U4 w = draw(p, env, 0, 0, D_INIT);
        t = 0.0 + p.inv_rate * std_exp(w.x, w.y);
    }
    p.t[env] = t;
    p.sc[env] = 0;
    p.topo[env] = 0;
    p.zcap[env] = 0;
    for (int w = 0; w < p.NZW; ++w) p.nzone[w * p.B + env] = 0;
    p.acc2[env] = 0;
    p.acc3[env] = 0;
    p.sum_lat[env] = 0;
    p.sum_cpu[env] = 0;
    p.sum_hi[env] = 0;
    p.total[env] = 0.0;
    p.last_r[env] = p.init_last_r;
}

// envs/baselines.py (:6-35): argmin topology latency / argmax zone cpu capacity / argmin
// endpoint cpu over feasible = mask[:-1] (masks are all True, :808-821), first index on
// ties (numpy); or a uniform random action keyed by (env, episode, step).  One lane/env.
__global__ void k_policy(Params p, int kind, int32_t* out) {
    int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= p.B) return;
    const Scal s = sc_unpack(p.sc[env]);
    if (kind == LB_POLICY_RANDOM) {
        out[env] = random_action(p, env, p.acc3[env], s.step);
        return;
    }
    const int nf = p.A - 1;
    if (nf <= 0) { out[env] = p.A - 1; return; }
    const uint64_t topo = p.topo[env], zc = p.zcap[env];
    double best = 0.0;
    int bi = 0;
    for (int e = 0; e < nf; ++e) {
        const int64_t i = eidx(p, env, e);
        const uint32_t em = p.emeta[i];
        double val;
        if (kind == LB_POLICY_TOPOLOGY_GREEDY) val = (double)topo_val(topo, em_zone(em), s.rz);
        else if (kind == LB_POLICY_ZONE_CPU_GREEDY) val = -(double)zcap_val(zc, em_zone(em));
        else val = cpu_of(p, em, p.edyn[i]);
        if (e == 0 || val < best) { best = val; bi = e; }
    }
    out[env] = bi;
}

__global__ void k_field(Params p, int field, double* out) {
    int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= p.B) return;
    const Scal s = sc_unpack(p.sc[env]);
    switch (field) {
    case LB_FIELD_CURRENT_TIME: out[env] = p.t[env]; return;
    case LB_FIELD_CURRENT_STEP: out[env] = (double)s.step; return;
    case LB_FIELD_REQUEST_ZONE: out[env] = (double)s.rz; return;
    case LB_FIELD_REQUEST_THRESHOLD: out[env] = (double)threshold(s.thr_idx); return;
    default: break;
    }
    const uint64_t topo = p.topo[env], zc = p.zcap[env];
    for (int e = 0; e < p.E; ++e) {
        const int64_t i = eidx(p, env, e);
        const uint32_t em = p.emeta[i], ed = p.edyn[i];
        double v;
        switch (field) {
        case LB_FIELD_ENDPOINT_LATENCY: v = lat_of(p, p.lat0[i], ed); break;
        case LB_FIELD_ENDPOINT_CPU: v = cpu_of(p, em, ed); break;
        case LB_FIELD_ENDPOINT_TOPOLOGY_LATENCY: v = (double)topo_val(topo, em_zone(em), s.rz); break;
        case LB_FIELD_ENDPOINT_ZONE_CPU_CAPACITY: v = (double)zcap_val(zc, em_zone(em)); break;
        case LB_FIELD_ENDPOINT_ZONE: v = (double)em_zone(em); break;
        case LB_FIELD_ENDPOINT_NODE: v = (double)em_node(em); break;
        default: v = (double)ed_j(ed); break;  // LB_FIELD_LOAD_SERVED
        }
        out[env * p.E + e] = v;
    }
}

__global__ void k_stats(Params p, double* out) {
    int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= p.B) return;
    write_stats_row(p, out + env * LB_ST_K, sc_unpack(p.sc[env]), p.acc2[env], p.acc3[env], p.total[env],
                    p.sum_lat[env], p.sum_cpu[env], p.sum_hi[env]);
}

__global__ void k_status(Params p, uint32_t* flags) {
    int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t f = 0;
    if (env < p.B) {
        Scal s = sc_unpack(p.sc[env]);
        if (s.bad) f |= LB_STATUS_BAD_ACTION;
        if (!s.reset_done) f |= LB_STATUS_NOT_RESET;
    }
    if (f) atomicOr(flags, f);
}

// ---- host side ---------------------------------------------------------------------------
thread_local std::string g_err;
#ifdef LB_EXPERIMENTS
// experiment switch of a diagnostic build (-DLB_EXPERIMENTS; lbx_set_rollout_variant,
// tools/roll_variants.py): 1 = k_rollout_img where k_rollout_lean would run, 3 = k_rollout_tpe
// for every L >= K launch (A/B references)
int g_rollout_variant = 0;
#else
constexpr int g_rollout_variant = 0;
#endif

int fail(const char* msg) {
    g_err = msg;
    return -1;
}

struct Geo {
    bool tpe;       // thread-per-env path (E <= 8)
    int W, EPL, EP, NZW;
};

// E > 8: W-lane slices.  Few envs (B < 32768): one env per wave (W = 16/32/64 by E), so
// the launch still has thousands of waves; many envs: 4 envs per wave up to E = 64, so
// the per-env scalar chain (Philox, logs, reward) is issued once per 4 envs and 4x more
// envs are in flight per CU.  Measured at E = 64 (A/B builds, profiles/r01_ablation.jsonl): 2^20 envs 1.45 ->
// 1.00 ms per step, 4096 envs 8.9 vs 20.7 us.  Both shapes give the same EP = W * EPL
// (the next power of two >= max(E, 16)), so the state layout does not depend on B.
constexpr int64_t WIDE_SLICE_MAX_B = 32768;
// E <= 8, few envs (config 2: 4096): 64-thread blocks, so the batch spreads over 4x more
// CUs (every TPE kernel works per wave).
constexpr int64_t SMALL_TPE_MAX_B = 65536;

Geo geometry(const lb_config* c, int64_t B = 0) {
    Geo g;
    const int E = c->num_endpoints;
    // E <= 8: one lane per env, except few envs (B < 32768, config 2), where lanes over
    // endpoints (the wide slice shape) cut each wave's serial chain: 4096 default envs
    // 10.8 -> 7.4 us per lb_step (A/B builds, profiles/r01_ablation.jsonl).
    // cfg->geometry pins the choice for E <= 8 (the state layout follows it).
    g.tpe = E <= TPE_E;
    if (g.tpe && B > 0 && B < WIDE_SLICE_MAX_B) g.tpe = false;
    if (E <= TPE_E && c->geometry == LB_GEOMETRY_TPE) g.tpe = true;
    if (c->geometry == LB_GEOMETRY_SLICE) g.tpe = false;
    if (g.tpe) {
        g.W = 1;
        g.EPL = 1;
        g.EP = E;
    } else {
        const bool wide = B < WIDE_SLICE_MAX_B;
        if (wide) {
            g.W = E <= 16 ? 16 : E <= 32 ? 32 : 64;
            g.EPL = E <= 64 ? 1 : E <= 128 ? 2 : 4;
        } else {
            g.W = E <= 64 ? 16 : E <= 128 ? 32 : 64;
            g.EPL = E <= 16 ? 1 : E <= 32 ? 2 : 4;
        }
        g.EP = g.W * g.EPL;
    }
    g.NZW = (c->num_nodes + 31) / 32;
    return g;
}

uint64_t align_up(uint64_t x) { return (x + 255) & ~(uint64_t)255; }

struct Offsets {
    uint64_t lat_lut, cpu_lut, lat0, emeta, edyn, t, sc, topo, zcap, nzone, acc2, acc3, sum_lat,
        sum_cpu, sum_hi, total, last_r, rew64, rec, end;
};

Offsets offsets(const lb_config* c, int64_t B) {
    Geo g = geometry(c, B);
    Offsets o;
    uint64_t x = 0;
    auto take = [&](uint64_t bytes) { uint64_t r = x; x = align_up(x + bytes); return r; };
    o.lat_lut = take((uint64_t)LAT_ROWS * JCAP * 8);
    o.cpu_lut = take((uint64_t)CPU_ROWS * JCAP * 8);
    const uint64_t BE = (uint64_t)B * g.EP;
    o.lat0 = take(BE * 8);
    o.emeta = take(BE * 4);
    o.edyn = take(BE * 4);
    o.t = take(B * 8);
    o.sc = take(B * 8);
    o.topo = take(B * 8);
    o.zcap = take(B * 8);
    o.nzone = take((uint64_t)B * g.NZW * 8);
    o.acc2 = take(B * 8);
    o.acc3 = take(B * 8);
    o.sum_lat = take(B * 8);
    o.sum_cpu = take(B * 8);
    o.sum_hi = take(B * 4);
    o.total = take(B * 8);
    o.last_r = take(B * 8);
    o.rew64 = take(B * 8);
    // thread-per-env layout: k_rollout_tpe's next-episode records (scratch, per launch)
    o.rec = take(g.tpe ? (uint64_t)B * RO_REC_BYTES : 0);
    o.end = x;
    return o;
}

double initial_last_reward(const lb_config* c) {
    // get_reward() right after reset(): penalty False, selected latency 0.0, topology 0.0,
    // cpu 1.0, all loads 0 (:297-327) — what an unrecognised first action returns.
    switch (c->reward_fn) {
    case LB_REWARD_NAIVE: return 1.0;
    case LB_REWARD_LATENCY: return -(0.0 + 0.0);
    case LB_REWARD_FAIRNESS: return 1.0 - 0.0;
    default: {
        volatile double cur = ((0.0 + 0.0) - 2.0) / 998.0;
        volatile double cpu = (1.0 - 1.0) / 99.0;
        volatile double a = c->latency_weight * (1.0 - cur);
        volatile double b = c->cpu_weight * (1.0 - cpu);
        volatile double g = c->gini_weight * (1.0 - 0.0);
        volatile double ab = a + b;
        return ab + g;
    }
    }
}

int validate(const lb_config* c) {
    if (!c) return fail("lb_config is NULL");
    if (c->num_endpoints < 1 || c->num_endpoints > EMAX) return fail("num_endpoints must be in [1, 256]");
    if (c->num_zones < 4)
        return fail("IndexError: num_zones < 4 (zone ids are drawn in [0,4), loadbalancer_k8s_env.py:354)");
    if (c->num_nodes < 24)
        return fail("IndexError: num_nodes < 24 (endpoint hosts are drawn in [0,24), loadbalancer_k8s_env.py:380)");
    if (c->num_nodes > 32 * NZW_MAX) return fail("num_nodes must be <= 256");
    if (c->episode_length < 1 || c->episode_length > CMAX) return fail("episode_length must be in [1, 1023]");
    if (c->reward_fn < 0 || c->reward_fn > 3) return fail("unknown reward_fn");
    if (c->rng_mode != LB_RNG_PHILOX && c->rng_mode != LB_RNG_TRACE) return fail("unknown rng_mode");
    if (c->geometry < LB_GEOMETRY_AUTO || c->geometry > LB_GEOMETRY_SLICE) return fail("unknown geometry");
    if (!(c->arrival_rate > 0.0)) return fail("arrival_rate must be > 0");
    return 0;
}

Params make_params(void* state, const lb_config* c, int64_t B) {
    Geo g = geometry(c, B);
    Offsets o = offsets(c, B);
    char* base = (char*)state;
    Params p;
    memset(&p, 0, sizeof(p));
    p.lat_lut = (double*)(base + o.lat_lut);
    p.cpu_lut = (double*)(base + o.cpu_lut);
    p.lat0 = (double*)(base + o.lat0);
    p.emeta = (uint32_t*)(base + o.emeta);
    p.edyn = (uint32_t*)(base + o.edyn);
    p.t = (double*)(base + o.t);
    p.sc = (uint64_t*)(base + o.sc);
    p.topo = (uint64_t*)(base + o.topo);
    p.zcap = (uint64_t*)(base + o.zcap);
    p.nzone = (uint64_t*)(base + o.nzone);
    p.acc2 = (uint64_t*)(base + o.acc2);
    p.acc3 = (uint64_t*)(base + o.acc3);
    p.sum_lat = (uint64_t*)(base + o.sum_lat);
    p.sum_cpu = (uint64_t*)(base + o.sum_cpu);
    p.sum_hi = (uint32_t*)(base + o.sum_hi);
    p.total = (double*)(base + o.total);
    p.last_r = (double*)(base + o.last_r);
    p.rew64 = (double*)(base + o.rew64);
    p.rec = g.tpe ? (uint4*)(base + o.rec) : nullptr;
    p.B = B;
    p.env_id_offset = c->env_id_offset;
    p.es = g.tpe ? B : 1;
    p.ee = g.tpe ? 1 : g.EP;
    p.E = c->num_endpoints;
    p.Z = c->num_zones;
    p.N = c->num_nodes;
    p.L = c->episode_length;
    p.R = c->num_endpoints + (c->rejection_allowed ? 1 : 0);
    p.A = p.R;
    p.EP = g.EP;
    p.NZW = g.NZW;
    p.reward_fn = c->reward_fn;
    p.rejection = c->rejection_allowed ? 1 : 0;
    p.auto_reset = c->auto_reset ? 1 : 0;
    p.inv_rate = 1.0 / c->arrival_rate;
    p.call = c->call_duration;
    p.lw = c->latency_weight;
    p.cw = c->cpu_weight;
    p.gw = c->gini_weight;
    p.init_last_r = initial_last_reward(c);
    p.key0 = (uint32_t)c->seed;
    p.key1 = (uint32_t)(c->seed >> 32);
    return p;
}

int check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = std::string("HIP launch failed: ") + hipGetErrorString(e);
        return -2;
    }
    return 0;
}

#define LB_DISPATCH_SLICE(W_, EPL_, BODY)                                         \
    do {                                                                          \
        if (W_ == 16 && EPL_ == 1) { constexpr int W = 16, EPL = 1; BODY; }       \
        else if (W_ == 16 && EPL_ == 2) { constexpr int W = 16, EPL = 2; BODY; }  \
        else if (W_ == 16 && EPL_ == 4) { constexpr int W = 16, EPL = 4; BODY; }  \
        else if (W_ == 32 && EPL_ == 4) { constexpr int W = 32, EPL = 4; BODY; }  \
        else if (W_ == 32 && EPL_ == 1) { constexpr int W = 32, EPL = 1; BODY; }  \
        else if (W_ == 64 && EPL_ == 1) { constexpr int W = 64, EPL = 1; BODY; }  \
        else if (W_ == 64 && EPL_ == 2) { constexpr int W = 64, EPL = 2; BODY; }  \
        else if (W_ == 64 && EPL_ == 4) { constexpr int W = 64, EPL = 4; BODY; }  \
        else return fail("unsupported geometry");                                 \
    } while (0)

unsigned slice_blocks(int64_t B, int W) {
    int64_t per = BLOCK / W;
    return (unsigned)((B + per - 1) / per);
}
unsigned env_blocks(int64_t B) { return (unsigned)((B + BLOCK - 1) / BLOCK); }

int device_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
    }
    return cus;
}

// Which kernel lb_rollout launches (lb_rollout_kernel reports it, LB_ROLLOUT_*).
// Per-lane addresses of the thread-per-env rollouts are 32-bit byte offsets from scalar bases
// (k_rollout_img: the state blob and the ep_stats rows; k_rollout_lean also the obs slot and
// the terminal observations), so they run only while every such offset fits in 32 bits; larger
// launches take k_rollout_tpe, which indexes in 64 bits.
int rollout_kernel(const lb_config* c, int64_t B, int32_t steps, bool outputs_all) {
    const Geo g = geometry(c, B);
    if (!g.tpe) return LB_ROLLOUT_SLICE;
    if (g.NZW > 2) return LB_ROLLOUT_STEPS;
    const bool pre = c->auto_reset && c->episode_length >= steps;
    if (!pre) return LB_ROLLOUT_TPE;
    const uint64_t lim = 0xFFFFFFFFull;
    const int R = c->num_endpoints + (c->rejection_allowed ? 1 : 0);
    const bool img_fits = offsets(c, B).end <= lim && (uint64_t)B * LB_ST_K * 8 <= lim;
    const bool lean_fits = img_fits && (uint64_t)B * R * 32 <= lim;
    const bool lean_shape = (c->num_endpoints == 8 && R == 9 && c->num_nodes <= 32) ||
                            (c->num_endpoints == 6 && R == 7 && c->num_nodes <= 64);
    if (lean_fits && lean_shape && B % 64 == 0 && B > SMALL_TPE_MAX_B && outputs_all &&
        g_rollout_variant == 0)
        return steps <= LEAN_SPLIT_MAX_K ? LB_ROLLOUT_LEAN_SPLIT : LB_ROLLOUT_LEAN;
    if (img_fits && g_rollout_variant != 3) return LB_ROLLOUT_IMG;
    return LB_ROLLOUT_TPE;
}

}  // namespace lbk

using namespace lbk;

extern "C" {

int lb_abi_version(void) { return LBK8S_ABI_VERSION; }

// (lb_source_hash, lb_build_flags, lb_build_compiler: lbk8s_build.cpp, rebuilt with every source change)

#ifdef LB_EXPERIMENTS
int lbx_set_rollout_variant(int v) { g_rollout_variant = v; return 0; }
#endif
#ifdef LB_TIMELINE
int lbx_set_timeline(uint64_t* buf) {  // k_rollout_img's (this unit) and k_rollout_lean's (one per policy unit)
    int r = hipMemcpyToSymbol(HIP_SYMBOL(g_timeline), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
    r |= lbx_set_timeline_lean_0(buf) | lbx_set_timeline_lean_1(buf) | lbx_set_timeline_lean_2(buf) |
         lbx_set_timeline_lean_3(buf);
    return r;
}
#endif

const char* lb_last_error(void) { return g_err.c_str(); }

int lb_validate_config(const lb_config* cfg) { return validate(cfg); }

int lb_state_bytes(const lb_config* cfg, int64_t num_envs, uint64_t* out_bytes) {
    if (int r = validate(cfg)) return r;
    if (num_envs < 1 || !out_bytes) return fail("num_envs must be >= 1 and out_bytes non-NULL");
    *out_bytes = offsets(cfg, num_envs).end;
    return 0;
}

int lb_init(void* state, const lb_config* cfg, int64_t num_envs, const lb_trace* trace, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || num_envs < 1) return fail("state NULL or num_envs < 1");
    const bool tr = cfg->rng_mode == LB_RNG_TRACE;
    if (tr && (!trace || !trace->t0)) return fail("trace mode: lb_init needs trace->t0");
    Params p = make_params(state, cfg, num_envs);
    if (tr) p.tr = *trace;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_luts, dim3((LAT_ROWS + CPU_ROWS + 127) / 128), dim3(128), 0, s, p.lat_lut, p.cpu_lut);
    if (int r = check_launch()) return r;
    hipLaunchKernelGGL(k_init, dim3(env_blocks(num_envs)), dim3(BLOCK), 0, s, p, tr ? 1 : 0);
    return check_launch();
}

int lb_reset(void* state, const lb_config* cfg, int64_t num_envs, const uint8_t* reset_mask,
             float* obs_out, const lb_trace* trace, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || num_envs < 1) return fail("state NULL or num_envs < 1");
    const bool tr = cfg->rng_mode == LB_RNG_TRACE;
    if (tr && (!trace || !trace->reset_lat0 || !trace->reset_topo || !trace->reset_ntype ||
               !trace->reset_nzone || !trace->reset_ncpu || !trace->reset_enode || !trace->reset_x1 ||
               !trace->reset_x2 || !trace->reset_r || !trace->reset_n))
        return fail("trace mode: lb_reset needs every reset_* trace array");
    Params p = make_params(state, cfg, num_envs);
    if (tr) p.tr = *trace;
    p.obs = obs_out;
    p.reset_mask = reset_mask;
    Geo g = geometry(cfg, num_envs);
    hipStream_t s = (hipStream_t)stream;
    if (g.tpe) {
        if (num_envs <= SMALL_TPE_MAX_B) {
            const unsigned nb = (unsigned)((num_envs + 63) / 64);
            if (tr) hipLaunchKernelGGL((k_reset_tpe<true, 64>), dim3(nb), dim3(64), 0, s, p);
            else hipLaunchKernelGGL((k_reset_tpe<false, 64>), dim3(nb), dim3(64), 0, s, p);
            return check_launch();
        }
        if (tr) hipLaunchKernelGGL(k_reset_tpe<true>, dim3(env_blocks(num_envs)), dim3(BLOCK), 0, s, p);
        else hipLaunchKernelGGL(k_reset_tpe<false>, dim3(env_blocks(num_envs)), dim3(BLOCK), 0, s, p);
        return check_launch();
    }
    LB_DISPATCH_SLICE(g.W, g.EPL, {
        if (tr) hipLaunchKernelGGL((k_reset_slice<W, EPL, true>), dim3(slice_blocks(num_envs, W)), dim3(BLOCK), 0, s, p);
        else hipLaunchKernelGGL((k_reset_slice<W, EPL, false>), dim3(slice_blocks(num_envs, W)), dim3(BLOCK), 0, s, p);
    });
    return check_launch();
}

int lb_step(void* state, const lb_config* cfg, int64_t num_envs, const int32_t* actions,
            float* obs_out, float* reward_out, uint8_t* done_out, float* terminal_obs_out,
            double* ep_stats_out, const lb_trace* trace, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || num_envs < 1) return fail("state NULL or num_envs < 1");
    const bool tr = cfg->rng_mode == LB_RNG_TRACE;
    if (!actions && tr) return fail("actions NULL (the fused random policy) needs Philox mode");
    if (tr && (!trace || !trace->step_x1 || !trace->step_x2 || !trace->step_r || !trace->step_n))
        return fail("trace mode: lb_step needs trace->step_* arrays");
    if (tr && cfg->auto_reset &&
        (!trace->reset_lat0 || !trace->reset_topo || !trace->reset_ntype || !trace->reset_nzone ||
         !trace->reset_ncpu || !trace->reset_enode || !trace->reset_x1 || !trace->reset_x2 ||
         !trace->reset_r || !trace->reset_n))
        return fail("trace mode with auto_reset: lb_step needs the reset_* arrays (any step may end an episode)");
    Params p = make_params(state, cfg, num_envs);
    if (tr) p.tr = *trace;
    p.actions = actions;
    p.obs = obs_out;
    p.reward = reward_out;
    p.done = done_out;
    p.term_obs = terminal_obs_out;
    p.ep_stats = ep_stats_out;
    Geo g = geometry(cfg, num_envs);
    hipStream_t s = (hipStream_t)stream;
    if (g.tpe) {
        // auto-reset (the finishing envs' reset()) runs inside k_step_tpe
        const bool recompute = !tr && num_envs >= SCEN_RECOMPUTE_MIN_B;
        if (num_envs <= SMALL_TPE_MAX_B && !recompute) {
            const unsigned nb = (unsigned)((num_envs + 63) / 64);
            if (tr) hipLaunchKernelGGL((k_step_tpe<true, false, 64>), dim3(nb), dim3(64), 0, s, p);
            else hipLaunchKernelGGL((k_step_tpe<false, false, 64>), dim3(nb), dim3(64), 0, s, p);
        } else if (tr) {
            hipLaunchKernelGGL((k_step_tpe<true, false>), dim3(env_blocks(num_envs)), dim3(BLOCK), 0, s, p);
        } else if (recompute) {
            hipLaunchKernelGGL((k_step_tpe<false, true>), dim3(env_blocks(num_envs)), dim3(BLOCK), 0, s, p);
        } else {
            hipLaunchKernelGGL((k_step_tpe<false, false>), dim3(env_blocks(num_envs)), dim3(BLOCK), 0, s, p);
        }
        return check_launch();
    }
    LB_DISPATCH_SLICE(g.W, g.EPL, {
        const unsigned nb = slice_blocks(num_envs, W);
        if (tr) hipLaunchKernelGGL((k_step_slice<W, EPL, true>), dim3(nb), dim3(BLOCK), 0, s, p);
        else hipLaunchKernelGGL((k_step_slice<W, EPL, false>), dim3(nb), dim3(BLOCK), 0, s, p);
    });
    return check_launch();
}

int lb_reward64(void* state, const lb_config* cfg, int64_t num_envs, double** out) {
    if (int r = validate(cfg)) return r;
    if (!state || num_envs < 1 || !out) return fail("state/out NULL or num_envs < 1");
    *out = make_params(state, cfg, num_envs).rew64;
    return 0;
}

int lb_rollout_kernel(const lb_config* cfg, int64_t num_envs, int32_t steps, int32_t outputs_all,
                      int32_t* kernel_out) {
    if (int r = validate(cfg)) return r;
    if (num_envs < 1 || steps < 0 || !kernel_out) return fail("num_envs < 1, steps < 0 or kernel_out NULL");
    // (lb_rollout's own preconditions: a launch it would reject has no kernel to name)
    if (cfg->rng_mode != LB_RNG_PHILOX) return fail("lb_rollout draws in Philox mode only");
    *kernel_out = rollout_kernel(cfg, num_envs, steps, outputs_all != 0);
    return 0;
}

int lb_rollout(void* state, const lb_config* cfg, int64_t num_envs, int32_t policy, int32_t steps,
               float* obs_out, float* reward_out, uint8_t* done_out, int32_t* actions_out,
               float* terminal_obs_out, double* ep_stats_out, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || num_envs < 1) return fail("state NULL or num_envs < 1");
    if (cfg->rng_mode != LB_RNG_PHILOX) return fail("lb_rollout draws in Philox mode only");
    if (policy < 0 || policy > LB_POLICY_RANDOM) return fail("unknown policy kind");
    if (steps < 0) return fail("steps must be >= 0");
    Geo g = geometry(cfg, num_envs);
    hipStream_t s = (hipStream_t)stream;
    if (g.tpe && g.NZW <= 2) {  // thread-per-env layout, N <= 64: K steps in one launch
        Params p = make_params(state, cfg, num_envs);
        p.obs = obs_out;
        p.reward = reward_out;
        p.done = done_out;
        p.term_obs = terminal_obs_out;
        p.ep_stats = ep_stats_out;
        const bool small = num_envs <= SMALL_TPE_MAX_B;
        const dim3 grid(small ? (unsigned)((num_envs + 63) / 64) : env_blocks(num_envs)), block(small ? 64 : BLOCK);
        // episodes at least as long as the launch (an env ends at most once in it): next
        // episodes drawn before the first step
        const bool pre = cfg->auto_reset && cfg->episode_length >= steps;
        const int rk = rollout_kernel(cfg, num_envs, steps, obs_out && reward_out && done_out && terminal_obs_out &&
                                                                ep_stats_out);
        if (rk == LB_ROLLOUT_LEAN || rk == LB_ROLLOUT_LEAN_SPLIT) {  // k_rollout_lean(_split) (lbk8s_lean.h), B % 64 == 0
            const bool e8 = p.E == 8, naive = p.reward_fn == LB_REWARD_NAIVE, act = actions_out != nullptr;
#define LB_LEAN(KIND_, ET_, RT_, NZW_)                                                                           \
            if (naive && act) launch_lean<KIND_, ET_, RT_, NZW_, true, true>(p, num_envs, (int)steps, actions_out, s); \
            else if (naive) launch_lean<KIND_, ET_, RT_, NZW_, true, false>(p, num_envs, (int)steps, actions_out, s); \
            else if (act) launch_lean<KIND_, ET_, RT_, NZW_, false, true>(p, num_envs, (int)steps, actions_out, s); \
            else launch_lean<KIND_, ET_, RT_, NZW_, false, false>(p, num_envs, (int)steps, actions_out, s);
#define LB_LEAN_KIND(KIND_) if (e8) { LB_LEAN(KIND_, 8, 9, 1) } else { LB_LEAN(KIND_, 6, 7, 2) }
            switch (policy) {
            case LB_POLICY_TOPOLOGY_GREEDY: LB_LEAN_KIND(LB_POLICY_TOPOLOGY_GREEDY); break;
            case LB_POLICY_ZONE_CPU_GREEDY: LB_LEAN_KIND(LB_POLICY_ZONE_CPU_GREEDY); break;
            case LB_POLICY_ENDPOINT_CPU_GREEDY: LB_LEAN_KIND(LB_POLICY_ENDPOINT_CPU_GREEDY); break;
            default: LB_LEAN_KIND(LB_POLICY_RANDOM); break;
            }
#undef LB_LEAN_KIND
#undef LB_LEAN
            return check_launch();
        }
        if (rk == LB_ROLLOUT_IMG) {  // k_rollout_img (lbk8s_rollout.h)
            const bool e8 = p.E == 8 && p.R == 9;
#define LB_IMG(NB_, KIND_)                                                                                   \
            if (e8) hipLaunchKernelGGL((k_rollout_img<NB_, KIND_, 8, 9, 4>), grid, block, 0, s, p, (int)steps, actions_out); \
            else hipLaunchKernelGGL((k_rollout_img<NB_, KIND_, 0, 0, 4>), grid, block, 0, s, p, (int)steps, actions_out);
#define LB_IMG_KIND(KIND_) if (small) { LB_IMG(64, KIND_) } else { LB_IMG(BLOCK, KIND_) }
            switch (policy) {
            case LB_POLICY_TOPOLOGY_GREEDY: LB_IMG_KIND(LB_POLICY_TOPOLOGY_GREEDY); break;
            case LB_POLICY_ZONE_CPU_GREEDY: LB_IMG_KIND(LB_POLICY_ZONE_CPU_GREEDY); break;
            case LB_POLICY_ENDPOINT_CPU_GREEDY: LB_IMG_KIND(LB_POLICY_ENDPOINT_CPU_GREEDY); break;
            default: LB_IMG_KIND(LB_POLICY_RANDOM); break;
            }
#undef LB_IMG_KIND
#undef LB_IMG
            return check_launch();
        }
#define LB_TPE_NB(NB_, KIND_)                                                                         \
        if (pre) hipLaunchKernelGGL((k_rollout_tpe<NB_, KIND_, true>), grid, block, 0, s, p, (int)steps, actions_out); \
        else hipLaunchKernelGGL((k_rollout_tpe<NB_, KIND_, false>), grid, block, 0, s, p, (int)steps, actions_out);
#define LB_TPE_KIND(KIND_)                         \
        if (small) { LB_TPE_NB(64, KIND_) }   \
        else { LB_TPE_NB(BLOCK, KIND_) }
        switch (policy) {
        case LB_POLICY_TOPOLOGY_GREEDY: LB_TPE_KIND(LB_POLICY_TOPOLOGY_GREEDY); break;
        case LB_POLICY_ZONE_CPU_GREEDY: LB_TPE_KIND(LB_POLICY_ZONE_CPU_GREEDY); break;
        case LB_POLICY_ENDPOINT_CPU_GREEDY: LB_TPE_KIND(LB_POLICY_ENDPOINT_CPU_GREEDY); break;
        default: LB_TPE_KIND(LB_POLICY_RANDOM); break;
        }
#undef LB_TPE_KIND
#undef LB_TPE_NB
        return check_launch();
    }
    if (g.tpe) {  // thread-per-env layout, N > 64: K policy + step launches
        if (policy != LB_POLICY_RANDOM && !actions_out)
            return fail("lb_rollout on the thread-per-env layout needs actions_out for a greedy policy");
        const int64_t R = cfg->num_endpoints + (cfg->rejection_allowed ? 1 : 0);
        for (int k = 0; k < steps; ++k) {
            int32_t* act = actions_out ? actions_out + k * num_envs : nullptr;
            if (act)
                if (int r = lb_policy(state, cfg, num_envs, policy, act, stream)) return r;
            if (int r = lb_step(state, cfg, num_envs, act, obs_out ? obs_out + k * num_envs * R * 8 : nullptr,
                                reward_out ? reward_out + k * num_envs : nullptr,
                                done_out ? done_out + k * num_envs : nullptr, terminal_obs_out, ep_stats_out,
                                nullptr, stream))
                return r;
        }
        return 0;
    }
    Params p = make_params(state, cfg, num_envs);
    p.obs = obs_out;
    p.reward = reward_out;
    p.done = done_out;
    p.term_obs = terminal_obs_out;
    p.ep_stats = ep_stats_out;
    if (g.W == 16 && g.EPL == 4 && p.E == 64 && p.R == 65 && g.NZW == 1) {  // config 4's shape, compile-time
        const dim3 grid(slice_blocks(num_envs, 16));
#define LB_SL64(RF_) hipLaunchKernelGGL((k_rollout_slice<16, 4, 64, 65, 1, RF_>), grid, dim3(BLOCK), 0, s, p, \
                                        (int)policy, (int)steps, actions_out)
        switch (p.reward_fn) {
        case LB_REWARD_NAIVE: LB_SL64(LB_REWARD_NAIVE); break;
        case LB_REWARD_LATENCY: LB_SL64(LB_REWARD_LATENCY); break;
        case LB_REWARD_FAIRNESS: LB_SL64(LB_REWARD_FAIRNESS); break;
        default: LB_SL64(LB_REWARD_MULTI); break;
        }
#undef LB_SL64
        return check_launch();
    }
    LB_DISPATCH_SLICE(g.W, g.EPL, {
        hipLaunchKernelGGL((k_rollout_slice<W, EPL>), dim3(slice_blocks(num_envs, W)), dim3(BLOCK), 0, s, p,
                           (int)policy, (int)steps, actions_out);
    });
    return check_launch();
}

int lb_policy(const void* state, const lb_config* cfg, int64_t num_envs, int32_t kind,
              int32_t* actions_out, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || !actions_out || num_envs < 1) return fail("state/actions_out NULL");
    if (kind < 0 || kind > LB_POLICY_RANDOM) return fail("unknown policy kind");
    Params p = make_params(const_cast<void*>(state), cfg, num_envs);
    hipLaunchKernelGGL(k_policy, dim3(env_blocks(num_envs)), dim3(BLOCK), 0, (hipStream_t)stream, p, (int)kind,
                       actions_out);
    return check_launch();
}

int lb_get_field(const void* state, const lb_config* cfg, int64_t num_envs, int32_t field, double* out,
                 void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || !out || num_envs < 1) return fail("state/out NULL");
    if (field < 0 || field >= LB_FIELD_COUNT) return fail("unknown field");
    if (field == LB_FIELD_DT) return fail("dt is not stored (it only feeds obs column 7)");
    Params p = make_params(const_cast<void*>(state), cfg, num_envs);
    hipLaunchKernelGGL(k_field, dim3(env_blocks(num_envs)), dim3(BLOCK), 0, (hipStream_t)stream, p, (int)field, out);
    return check_launch();
}

int lb_get_stats(const void* state, const lb_config* cfg, int64_t num_envs, double* stats_out, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || !stats_out || num_envs < 1) return fail("state/stats_out NULL");
    Params p = make_params(const_cast<void*>(state), cfg, num_envs);
    hipLaunchKernelGGL(k_stats, dim3(env_blocks(num_envs)), dim3(BLOCK), 0, (hipStream_t)stream, p, stats_out);
    return check_launch();
}

int lb_status(const void* state, const lb_config* cfg, int64_t num_envs, uint32_t* flags_out, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!state || !flags_out || num_envs < 1) return fail("state/flags_out NULL");
    Params p = make_params(const_cast<void*>(state), cfg, num_envs);
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(flags_out, 0, sizeof(uint32_t), s) != hipSuccess) return fail("hipMemsetAsync failed");
    hipLaunchKernelGGL(k_status, dim3(env_blocks(num_envs)), dim3(BLOCK), 0, s, p, flags_out);
    return check_launch();
}

int lb_episode_log(int64_t num_envs, const uint8_t* done, const double* ep_stats, const float* reward,
                   const double* reward64, const int32_t* actions, float* ret32, float* ep_r32, int64_t tag, double* log, int64_t cap,
                   uint32_t* count, void* stream) {
    if (num_envs < 1 || !done || !ep_stats || !reward || !actions || !ret32 || !log || !count || cap < 0)
        return fail("episode log: buffers NULL or num_envs < 1");
    EpLogParams p{num_envs, done, ep_stats, reward, reward64, actions, ret32, ep_r32, tag, log, cap, count};
    hipLaunchKernelGGL(k_episode_log, dim3(env_blocks(num_envs)), dim3(BLOCK), 0, (hipStream_t)stream, p);
    return check_launch();
}

int lb_ds_pack(const lb_ds_weights* w, float* frag_out, void* stream) {
    if (!w || !frag_out) return fail("weights/frag_out NULL");
    for (int i = 0; i < 3; ++i)
        if (!w->actor_lambda[i] || !w->actor_gamma[i]) return fail("actor weights are required");
    hipLaunchKernelGGL(k_ds_pack, dim3((DS_IMG_FLOATS + 255) / 256), dim3(256), 0, (hipStream_t)stream, *w, frag_out);
    return check_launch();
}

}  // extern "C"

#ifndef LB_DS_WAVES_PER_SIMD
#define LB_DS_WAVES_PER_SIMD 1
#endif
namespace {
// persistent grid for the deep-sets kernels (the weight image is staged once per block)
unsigned ds_grid(int64_t groups) {
    const int64_t want = (groups + DS_BLOCK / 64 - 1) / (DS_BLOCK / 64);
    return (unsigned)std::min<int64_t>(want, device_cus());
}
// k_deepsets_fwd numbers its waves wave-major (wave w of block b = w * grid + b): every CU
// gets a block as soon as there are as many groups as CUs
unsigned ds_grid_spread(int64_t groups) { return (unsigned)std::min<int64_t>(groups, device_cus()); }

template <int MODE>
void ds_forward_launch(const DSParams& p, hipStream_t s) {
    if (p.R > LB_DS_MAX_ELEMENTS) {  // large sets: streamed in chunks, one env per wave
        hipLaunchKernelGGL((k_deepsets_fwd_big<MODE>), dim3(ds_grid(p.B)), dim3(DS_BLOCK), 0, s, p);
        return;
    }
    // a wave takes P envs per iteration: P = 4 for R <= 16, 2 for R <= 32, else 1 -- fewer
    // when the batch would leave SIMDs of the chip idle (the DQN vector step's 4096 envs:
    // 1,024 groups of four, one per SIMD; its 128-set train step)
    const int ts = (p.R + 15) / 16;
    // (the greedy-action forward of small sets takes at most two envs per iteration: its Gamma
    // terms on the VALU, the arithmetic of k_dqn_step's Q forward)
    int P = ts == 1 ? (MODE == 2 ? 2 : 4) : (ts == 2 ? 2 : 1);
    {
        const int64_t simds = (int64_t)device_cus() * 4 * LB_DS_WAVES_PER_SIMD;
        while (P > 1 && (p.B + P - 1) / P < simds) P /= 2;
    }
    const unsigned grid = ds_grid_spread((p.B + P - 1) / P);
    if constexpr (MODE == 1) {  // R = 16 TS + 1 (config 4's 65): TS tiles and the extra row (XR)
        if (p.R == 49) {
            hipLaunchKernelGGL((k_deepsets_fwd<3, 1, 1, true>), dim3(grid), dim3(DS_BLOCK), 0, s, p);
            return;
        }
        if (p.R == 65) {
            hipLaunchKernelGGL((k_deepsets_fwd<4, 1, 1, true>), dim3(grid), dim3(DS_BLOCK), 0, s, p);
            return;
        }
    }
    switch (ts) {
        case 1:
            if (P == 4) hipLaunchKernelGGL((k_deepsets_fwd<1, 4, MODE>), dim3(grid), dim3(DS_BLOCK), 0, s, p);
            else if (P == 2) hipLaunchKernelGGL((k_deepsets_fwd<1, 2, MODE>), dim3(grid), dim3(DS_BLOCK), 0, s, p);
            else hipLaunchKernelGGL((k_deepsets_fwd<1, 1, MODE>), dim3(grid), dim3(DS_BLOCK), 0, s, p);
            break;
        case 2:
            if (P == 2) hipLaunchKernelGGL((k_deepsets_fwd<2, 2, MODE>), dim3(grid), dim3(DS_BLOCK), 0, s, p);
            else hipLaunchKernelGGL((k_deepsets_fwd<2, 1, MODE>), dim3(grid), dim3(DS_BLOCK), 0, s, p);
            break;
        case 3: hipLaunchKernelGGL((k_deepsets_fwd<3, 1, MODE>), dim3(grid), dim3(DS_BLOCK), 0, s, p); break;
        case 4: hipLaunchKernelGGL((k_deepsets_fwd<4, 1, MODE>), dim3(grid), dim3(DS_BLOCK), 0, s, p); break;
        default: hipLaunchKernelGGL((k_deepsets_fwd<5, 1, MODE>), dim3(grid), dim3(DS_BLOCK), 0, s, p); break;
    }
}
}  // namespace

extern "C" {

int lb_ds_forward(const float* frag, const float* obs, int64_t num_envs, int32_t num_elements, float* logits_out,
                  float* value_out, void* stream) {
    static_assert(DS_IMG_FLOATS == LB_DS_FRAG_FLOATS, "weight image layout and header disagree");
    if (!frag || !obs || num_envs < 1) return fail("frag/obs NULL or num_envs < 1");
    if (num_elements < 1 || num_elements > LB_DS_MAX_ELEMENTS_FWD)
        return fail("num_elements must be in [1, 257] (LB_DS_MAX_ELEMENTS_FWD)");
    if (!logits_out && !value_out) return 0;
    DSParams p{obs, frag, logits_out, value_out, num_envs, num_elements, logits_out != nullptr, value_out != nullptr,
               nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    ds_forward_launch<0>(p, (hipStream_t)stream);
    return check_launch();
}

int lb_ds_q_argmax(const float* frag, const float* obs, int64_t num_envs, int32_t num_elements, const uint8_t* masks,
                   float* q_out, int32_t* actions_out, void* stream) {
    if (!frag || !obs || !actions_out || num_envs < 1) return fail("frag/obs/actions_out NULL or num_envs < 1");
    if (num_elements < 1 || num_elements > LB_DS_MAX_ELEMENTS_FWD)
        return fail("num_elements must be in [1, 257] (LB_DS_MAX_ELEMENTS_FWD)");
    DSParams p{obs, frag, q_out, nullptr, num_envs, num_elements, 1, 0, nullptr, nullptr, nullptr, nullptr, actions_out,
               masks};
    ds_forward_launch<2>(p, (hipStream_t)stream);
    return check_launch();
}

int lb_replay_add(int64_t num_envs, int32_t obs_floats, int64_t slots, const int64_t* pos_in, int64_t* pos_out,
                  float* obs, const float* next_obs, const int32_t* actions, const float* reward, const uint8_t* done,
                  const double* ep_stats, float* rb_obs, float* rb_next_obs, int64_t* rb_actions, float* rb_rewards,
                  float* rb_dones, double* ep_sum, double* ep_cnt, void* stream) {
    if (num_envs < 1 || obs_floats < 4 || obs_floats % 4 || slots < 1) return fail("bad replay geometry");
    if (!pos_in || !pos_out || pos_in == pos_out || !obs || !next_obs || !actions || !reward || !done || !rb_obs ||
        !rb_next_obs || !rb_actions || !rb_rewards || !rb_dones || ((ep_sum || ep_cnt) && !(ep_sum && ep_cnt && ep_stats)))
        return fail("replay buffers NULL (or pos_in == pos_out)");
    ReplayParams p{num_envs, obs_floats / 4, slots, pos_in, pos_out, reinterpret_cast<float4*>(obs),
                   reinterpret_cast<const float4*>(next_obs), actions, reward, done, ep_stats,
                   reinterpret_cast<float4*>(rb_obs), reinterpret_cast<float4*>(rb_next_obs), rb_actions, rb_rewards,
                   rb_dones, ep_sum, ep_cnt};
    const int64_t n = std::max<int64_t>(num_envs * p.f4, num_envs);
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 65535);
    hipLaunchKernelGGL(k_replay_add, dim3(grid), dim3(256), 0, (hipStream_t)stream, p);
    return check_launch();
}

int lb_dqn_act(const float* frag, const float* obs, int64_t num_envs, int32_t num_elements, const uint8_t* masks,
               const void* state, const lb_config* cfg, const lb_dqn_explore* ex, int32_t* actions_out,
               void* stream) {
    if (int r = validate(cfg)) return r;
    if (!frag || !obs || !state || !ex || !actions_out || num_envs < 1)
        return fail("frag/obs/state/ex/actions_out NULL or num_envs < 1");
    if (!ex->vstep_in || !ex->vstep_out || ex->vstep_in == ex->vstep_out || !ex->explore_out)
        return fail("lb_dqn_explore: device words NULL (or vstep_in == vstep_out)");
    if (cfg->rng_mode != LB_RNG_PHILOX) return fail("lb_dqn_act draws in Philox mode only");
    const int32_t A = cfg->num_endpoints + (cfg->rejection_allowed ? 1 : 0);
    if (num_elements != A) return fail("lb_dqn_act: num_elements must be the env's action count (R)");
    if (num_elements < 1 || num_elements > LB_DS_MAX_ELEMENTS_FWD)
        return fail("num_elements must be in [1, 257] (LB_DS_MAX_ELEMENTS_FWD)");
    const Params e = make_params(const_cast<void*>(state), cfg, num_envs);
    DSParams p{obs, frag, nullptr, nullptr, num_envs, num_elements, 1, 0, nullptr, nullptr, nullptr, nullptr,
               actions_out, masks};
    p.ex_on = 1;
    p.ex = *ex;
    p.ex_acc3 = e.acc3;
    p.ex_sc = e.sc;
    p.ex_env_offset = e.env_id_offset;
    p.ex_key0 = e.key0;
    p.ex_key1 = e.key1;
    ds_forward_launch<2>(p, (hipStream_t)stream);
    return check_launch();
}

namespace {
// lb_dqn_step's one-launch shape: the env in the slice layout with 16 lanes per env (E <= 16
// below 32,768 envs) and R <= 16.  A property of the shape only (not of the device's CU count):
// the kernel is correct for any number of envs, and the learner's path must not change with the
// part it runs on
bool dqn_step_fusable(const lb_config* cfg, int64_t num_envs, int32_t num_elements) {
    const Geo g = geometry(cfg, num_envs);
    return !g.tpe && g.W == 16 && g.EPL == 1 && num_elements <= 16;
}

int dqn_steps_launch(const float* frag, float* obs, int64_t num_envs, int32_t num_elements, const uint8_t* masks,
                     void* state, const lb_config* cfg, const lb_dqn_explore* ex, int32_t* actions_out,
                     float* next_obs_out, float* reward_out, uint8_t* done_out, float* terminal_obs_out,
                     double* ep_stats_out, int64_t slots, const int64_t* pos_in, int64_t* pos_out, float* rb_obs,
                     float* rb_next_obs, int64_t* rb_actions, float* rb_rewards, float* rb_dones, double* ep_sum,
                     double* ep_cnt, int32_t steps, int32_t* sync, void* stream) {
    // (the three entry points' checks)
    if (!frag || !obs || !state || !ex || !actions_out || !next_obs_out || !reward_out || !done_out || num_envs < 1)
        return fail("lb_dqn_step: frag/obs/state/ex/actions/next_obs/reward/done NULL or num_envs < 1");
    if (!ex->vstep_in || !ex->vstep_out || (!sync && ex->vstep_in == ex->vstep_out) || !ex->explore_out)
        return fail("lb_dqn_explore: device words NULL (or vstep_in == vstep_out)");
    if (cfg->rng_mode != LB_RNG_PHILOX) return fail("lb_dqn_step draws in Philox mode only");
    const int32_t A = cfg->num_endpoints + (cfg->rejection_allowed ? 1 : 0);
    if (num_elements != A) return fail("lb_dqn_step: num_elements must be the env's action count (R)");
    if (slots < 1 || !pos_in || !pos_out || (!sync && pos_in == pos_out) || !rb_obs || !rb_next_obs ||
        !rb_actions || !rb_rewards || !rb_dones || ((ep_sum || ep_cnt) && !(ep_sum && ep_cnt && ep_stats_out)))
        return fail("replay buffers NULL (or pos_in == pos_out)");
    Params e = make_params(state, cfg, num_envs);
    e.obs = next_obs_out;
    e.reward = reward_out;
    e.done = done_out;
    e.term_obs = terminal_obs_out;
    e.ep_stats = ep_stats_out;
    DSParams d{obs, frag, nullptr, nullptr, num_envs, num_elements, 1, 0, nullptr, nullptr, nullptr, nullptr,
               actions_out, masks};
    d.ex_on = 1;
    d.ex = *ex;
    d.ex_acc3 = e.acc3;
    d.ex_sc = e.sc;
    d.ex_env_offset = e.env_id_offset;
    d.ex_key0 = e.key0;
    d.ex_key1 = e.key1;
    DQNReplay r{slots, num_elements * 2, pos_in, pos_out, reinterpret_cast<float4*>(obs),
                reinterpret_cast<float4*>(rb_obs), reinterpret_cast<float4*>(rb_next_obs), rb_actions, rb_rewards,
                rb_dones, ep_sum, ep_cnt};
    constexpr int P = 2;  // envs per wave iteration: 2 puts the 4096-env batch on every wave of the grid (4: half the waves idle)
    const unsigned grid = ds_grid_spread((num_envs + P - 1) / P);
    hipLaunchKernelGGL(k_dqn_step<P>, dim3(grid), dim3(DS_BLOCK), 0, (hipStream_t)stream, d, e, r, (int)steps, sync);
    return check_launch();
}
}  // namespace

int lb_dqn_step(const float* frag, float* obs, int64_t num_envs, int32_t num_elements, const uint8_t* masks,
                void* state, const lb_config* cfg, const lb_dqn_explore* ex, int32_t* actions_out,
                float* next_obs_out, float* reward_out, uint8_t* done_out, float* terminal_obs_out,
                double* ep_stats_out, int64_t slots, const int64_t* pos_in, int64_t* pos_out, float* rb_obs,
                float* rb_next_obs, int64_t* rb_actions, float* rb_rewards, float* rb_dones, double* ep_sum,
                double* ep_cnt, void* stream) {
    if (int r = validate(cfg)) return r;
    if (!dqn_step_fusable(cfg, num_envs, num_elements)) {  // the three launches
        if (int rc = lb_dqn_act(frag, obs, num_envs, num_elements, masks, state, cfg, ex, actions_out, stream)) return rc;
        if (int rc = lb_step(state, cfg, num_envs, actions_out, next_obs_out, reward_out, done_out, terminal_obs_out,
                             ep_stats_out, nullptr, stream))
            return rc;
        return lb_replay_add(num_envs, num_elements * 8, slots, pos_in, pos_out, obs, next_obs_out, actions_out,
                             reward_out, done_out, ep_stats_out, rb_obs, rb_next_obs, rb_actions, rb_rewards, rb_dones,
                             ep_sum, ep_cnt, stream);
    }
    return dqn_steps_launch(frag, obs, num_envs, num_elements, masks, state, cfg, ex, actions_out, next_obs_out,
                            reward_out, done_out, terminal_obs_out, ep_stats_out, slots, pos_in, pos_out, rb_obs,
                            rb_next_obs, rb_actions, rb_rewards, rb_dones, ep_sum, ep_cnt, 1, nullptr, stream);
}

int lb_dqn_steps_supported(const lb_config* cfg, int64_t num_envs, int32_t num_elements) {
    if (validate(cfg)) return 0;
    return dqn_step_fusable(cfg, num_envs, num_elements) ? 1 : 0;
}

int lb_dqn_steps(const float* frag, float* obs, int64_t num_envs, int32_t num_elements, const uint8_t* masks,
                 void* state, const lb_config* cfg, const lb_dqn_explore* ex, int32_t* actions_out,
                 float* next_obs_out, float* reward_out, uint8_t* done_out, float* terminal_obs_out,
                 double* ep_stats_out, int64_t slots, const int64_t* pos_in, int64_t* pos_out, float* rb_obs,
                 float* rb_next_obs, int64_t* rb_actions, float* rb_rewards, float* rb_dones, double* ep_sum,
                 double* ep_cnt, int32_t steps, int32_t* sync, void* stream) {
    if (int r = validate(cfg)) return r;
    if (steps < 1 || steps > 32) return fail("lb_dqn_steps: steps must be in [1, 32]");
    if (!sync) return fail("lb_dqn_steps: sync (a device int32 that is 0) is required");
    if (!dqn_step_fusable(cfg, num_envs, num_elements))
        return fail("lb_dqn_steps: the env's shape has no one-launch vector step (lb_dqn_steps_supported)");
    return dqn_steps_launch(frag, obs, num_envs, num_elements, masks, state, cfg, ex, actions_out, next_obs_out,
                            reward_out, done_out, terminal_obs_out, ep_stats_out, slots, pos_in, pos_out, rb_obs,
                            rb_next_obs, rb_actions, rb_rewards, rb_dones, ep_sum, ep_cnt, steps, sync, stream);
}

int lb_dqn_head(const float* q, const float* q_next, const int64_t* actions, const float* rewards, const float* dones,
                int64_t num_sets, int32_t num_elements, float gamma, float* dq_out, float* sq_err_out, float* td_out,
                float* old_out, float* loss_out, void* stream) {
    if (!q || !q_next || !actions || !rewards || !dones || !dq_out || !sq_err_out || num_sets < 1)
        return fail("lb_dqn_head: NULL buffer or num_sets < 1");
    if (num_elements < 1 || num_elements > LB_DS_MAX_ELEMENTS_TRAIN) return fail("num_elements must be in [1, 257]");
    if (loss_out && num_sets > DQN_HEAD_BLOCK_MAX) return fail("lb_dqn_head: loss_out needs num_sets <= 1024");
    DQNHeadParams p{q, q_next, actions, rewards, dones, num_sets, num_elements, gamma, 2.0f / (float)num_sets, dq_out,
                    sq_err_out, td_out, old_out, loss_out};
    if (loss_out) {  // one block, one lane per sample, the mean in the same launch
        hipLaunchKernelGGL(k_dqn_head_block, dim3(1), dim3((unsigned)((num_sets + 63) / 64 * 64)), 0,
                           (hipStream_t)stream, p);
        return check_launch();
    }
    const unsigned grid = (unsigned)std::min<int64_t>((num_sets + 3) / 4, 65535);
    hipLaunchKernelGGL(k_dqn_head, dim3(grid), dim3(256), 0, (hipStream_t)stream, p);
    return check_launch();
}

int lb_replay_sample(int64_t num_envs, int32_t obs_floats, int64_t slots, int32_t batch, uint64_t seed,
                     const int64_t* vstep, const int64_t* base_adds, const float* rb_obs, const float* rb_next_obs,
                     const int64_t* rb_actions, const float* rb_rewards, const float* rb_dones, float* obs_out,
                     float* next_obs_out, int64_t* actions_out, float* rewards_out, float* dones_out, void* stream) {
    if (num_envs < 1 || obs_floats < 4 || obs_floats % 4 || slots < 1 || slots >= (1ll << 32) || batch < 1 ||
        num_envs >= (1ll << 32))
        return fail("bad replay sample geometry");
    if (!vstep || !base_adds || !rb_obs || !rb_next_obs || !rb_actions || !rb_rewards || !rb_dones || !obs_out ||
        !next_obs_out || !actions_out || !rewards_out || !dones_out)
        return fail("replay sample buffers NULL");
    ReplaySampleParams p{num_envs, obs_floats / 4, slots, batch, seed, vstep, base_adds,
                         reinterpret_cast<const float4*>(rb_obs), reinterpret_cast<const float4*>(rb_next_obs),
                         rb_actions, rb_rewards, rb_dones, reinterpret_cast<float4*>(obs_out),
                         reinterpret_cast<float4*>(next_obs_out), actions_out, rewards_out, dones_out};
    const int64_t n = (int64_t)batch * (2 * p.f4 + 1);
    hipLaunchKernelGGL(k_replay_sample, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, p);
    return check_launch();
}

int lb_ds_train_forward(const float* frag, const float* obs, int64_t num_envs, int32_t num_elements,
                        float* logits_out, float* psi_mean_out, float* save_actor, float* save_critic,
                        float* setvec_out, void* stream) {
    if (!frag || !obs || !setvec_out || num_envs < 1) return fail("frag/obs/setvec_out NULL or num_envs < 1");
    if (num_elements < 1 || num_elements > LB_DS_MAX_ELEMENTS_TRAIN)
        return fail("num_elements must be in [1, 257] (LB_DS_MAX_ELEMENTS_TRAIN)");
    if (!logits_out && !psi_mean_out) return 0;
    if ((logits_out && !save_actor) || (psi_mean_out && !save_critic))
        return fail("a head's activation buffer is NULL");
    DSParams p{obs, frag, logits_out, nullptr, num_envs, num_elements, logits_out != nullptr, psi_mean_out != nullptr,
               save_actor, save_critic, psi_mean_out, setvec_out, nullptr, nullptr};
    ds_forward_launch<1>(p, (hipStream_t)stream);
    return check_launch();
}

int lb_ds_forward_pair(const float* frag_a, const float* obs_a, float* logits_a, const float* frag_b,
                       const float* obs_b, float* logits_b, float* save_actor_b, float* setvec_b, int64_t num_envs,
                       int32_t num_elements, void* stream) {
    if (!frag_a || !obs_a || !logits_a || !frag_b || !obs_b || !logits_b || !save_actor_b || !setvec_b || num_envs < 1)
        return fail("lb_ds_forward_pair: NULL buffer or num_envs < 1");
    if (num_elements < 1 || num_elements > 16) return fail("lb_ds_forward_pair: num_elements must be in [1, 16]");
    DSParams a{obs_a, frag_a, logits_a, nullptr, num_envs, num_elements, 1, 0,
               nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    DSParams b{obs_b, frag_b, logits_b, nullptr, num_envs, num_elements, 1, 0,
               save_actor_b, nullptr, nullptr, setvec_b, nullptr, nullptr};
    // P as ds_forward_launch picks it for one of the two (the batch against the chip's SIMDs)
    int P = 4;
    {
        const int64_t simds = (int64_t)device_cus() * 4 * LB_DS_WAVES_PER_SIMD;
        while (P > 1 && (num_envs + P - 1) / P < simds) P /= 2;
    }
    const int ga = (int)ds_grid_spread((num_envs + P - 1) / P);
    const dim3 grid(2 * ga);
    if (P == 4) hipLaunchKernelGGL((k_ds_fwd_pair<1, 4>), grid, dim3(DS_BLOCK), 0, (hipStream_t)stream, a, b, ga);
    else if (P == 2) hipLaunchKernelGGL((k_ds_fwd_pair<1, 2>), grid, dim3(DS_BLOCK), 0, (hipStream_t)stream, a, b, ga);
    else hipLaunchKernelGGL((k_ds_fwd_pair<1, 1>), grid, dim3(DS_BLOCK), 0, (hipStream_t)stream, a, b, ga);
    return check_launch();
}

int lb_ppo_head(const float* logits, const uint8_t* masks, const float* actions, const float* oldlogp,
                const float* adv, const float* ret, const float* vold, const float* value, int64_t num_sets,
                int32_t num_elements, float clip_coef, float ent_coef, float vf_coef, int32_t clip_vloss,
                float* dlogits, float* dvalue, float* terms, void* stream) {
    if (!logits || !actions || !oldlogp || !adv || !ret || !vold || !value || !dlogits || !dvalue || !terms ||
        num_sets < 1)
        return fail("ppo head buffers NULL or num_sets < 1");
    if (num_elements < 1 || num_elements > LB_DS_MAX_ELEMENTS_TRAIN) return fail("num_elements must be in [1, 257]");
    PPOHeadParams p{logits, masks, actions, oldlogp, adv, ret, vold, value, dlogits, dvalue, terms,
                    num_sets, num_elements, clip_coef, ent_coef, vf_coef, 1.0f / (float)num_sets, clip_vloss};
    const unsigned grid = (unsigned)std::min<int64_t>((num_sets + 3) / 4, 8192);
    hipLaunchKernelGGL(k_ppo_head, dim3(grid), dim3(256), 0, (hipStream_t)stream, p);
    return check_launch();
}

int lb_ds_pack_backward(const lb_ds_weights* w, float* bwd_frag_out, void* stream) {
    static_assert(DSB_FLOATS == LB_DS_BWD_FLOATS, "backward image layout and header disagree");
    if (!w || !bwd_frag_out) return fail("weights/bwd_frag_out NULL");
    if (!w->actor_lambda[1] || !w->actor_gamma[1] || !w->actor_lambda[2] || !w->actor_gamma[2])
        return fail("actor weights are required");
    hipLaunchKernelGGL(k_ds_pack_bwd, dim3((DSB_FLOATS + 255) / 256), dim3(256), 0, (hipStream_t)stream, *w,
                       bwd_frag_out);
    return check_launch();
}

int lb_ds_pack_pair(const lb_ds_weights* w, float* frag_out, float* bwd_frag_out, void* stream) {
    if (!w || !frag_out || !bwd_frag_out) return fail("weights/frag_out/bwd_frag_out NULL");
    for (int i = 0; i < 3; ++i)
        if (!w->actor_lambda[i] || !w->actor_gamma[i]) return fail("actor weights are required");
    hipLaunchKernelGGL(k_ds_pack_pair, dim3(DS_PACK_BLOCKS + DSB_PACK_BLOCKS), dim3(256), 0, (hipStream_t)stream, *w,
                       frag_out, bwd_frag_out);
    return check_launch();
}

}  // extern "C"
namespace {
// lb_ds_set_grads' jobs (returns their count)
int set_grad_params(const float* setvec, const float* dlogits, const float* dmean, int64_t num_sets,
                    int32_t num_elements, float* out, SetGradParams& p) {
    const int SV = LB_DS_SETVEC_FLOATS;
    p = SetGradParams{};
    p.S = num_sets;
    int nj = 0;
    auto job = [&](const float* a, int lda, int M, int amode, int alen, int boff, const float* b, int ldb, int N,
                   float scale, float* o) {
        p.job[nj++] = SetGradJob{a, lda, M, amode, alen, b ? b : setvec + boff, ldb, N, scale, o};
    };
    // actor: dGamma1 = -GS1A^T MAX0, dGamma2 = -GS2A^T MAX1A, dLambda3 = sum GA3,
    // dGamma3 = -(row sums of dlogits)^T MAX2A
    job(setvec + LB_DSV_GS1A, SV, 64, 0, 0, LB_DSV_MAX0, nullptr, SV, 8, -1.f, out);
    job(setvec + LB_DSV_GS2A, SV, 64, 0, 0, LB_DSV_MAX1A, nullptr, SV, 64, -1.f, out + 512);
    job(nullptr, 0, 1, 1, 0, LB_DSV_GA3, nullptr, SV, 64, 1.f, out + 4608);
    job(dlogits, num_elements, 1, 2, num_elements, LB_DSV_MAX2A, nullptr, SV, 64, -1.f, out + 4672);
    if (dmean) {  // critic: the same for psi, layer 3 from dmean (the mean's 1/R on Lambda3)
        float* c = out + LB_DS_SETGRAD_ACTOR;
        job(setvec + LB_DSV_GS1C, SV, 64, 0, 0, LB_DSV_MAX0, nullptr, SV, 8, -1.f, c);
        job(setvec + LB_DSV_GS2C, SV, 64, 0, 0, LB_DSV_MAX1C, nullptr, SV, 64, -1.f, c + 512);
        job(dmean, 64, 64, 0, 0, LB_DSV_CS2, nullptr, SV, 64, 1.f / (float)num_elements, c + 4608);
        job(dmean, 64, 64, 0, 0, LB_DSV_MAX2C, nullptr, SV, 64, -1.f, c + 8704);
    }
    static_assert(LB_DS_SETGRAD_ACTOR == 4736 && LB_DS_SETGRAD_CRITIC == 12800, "set-gradient layout");
    return nj;
}
// the training backward's launches (set_grads_out: lb_ds_train_backward_sets)
int train_backward(const float* bwd_frag, const float* obs, int64_t num_envs, int32_t num_elements,
                   const float* save_actor, const float* save_critic, const float* dlogits, const float* dmean,
                   float* wgrad_out, float* workspace, float* setvec, float* set_grads_out, void* stream) {
    static_assert(DSV_FLOATS == LB_DS_SETVEC_FLOATS, "per-set vector layout and header disagree");
    static_assert(DSW_FLOATS == LB_DS_WGRAD_FLOATS && DSW_SLOTS * 2 * DSW_FLOATS <= LB_DS_WORKSPACE_FLOATS,
                  "weight-gradient layout and header disagree");
    if (!bwd_frag || !obs || !setvec || !wgrad_out || !workspace || num_envs < 1)
        return fail("bwd_frag/obs/setvec/wgrad_out/workspace NULL or num_envs < 1");
    if (num_elements < 1 || num_elements > LB_DS_MAX_ELEMENTS_TRAIN)
        return fail("num_elements must be in [1, 257] (LB_DS_MAX_ELEMENTS_TRAIN)");
    const bool actor = dlogits != nullptr, critic = dmean != nullptr;
    if ((actor && !save_actor) || (critic && !save_critic)) return fail("a head's activation buffer is NULL");
    DSBwdParams p{obs, bwd_frag, save_actor, save_critic, dlogits, dmean, workspace, setvec,
                  num_envs, num_elements, actor, critic};
    // fixed grid: one workspace slot per block, so the reduction order never depends on B
    hipStream_t s = (hipStream_t)stream;
    // each head's backward (layer 1's pooled term in its slots too)
    if (actor) {
        hipLaunchKernelGGL(k_ds_train_bwd<0>, dim3(DSW_GRID), dim3(DSB_BLOCK), 0, s, p);
        if (int r = check_launch()) return r;
    }
    if (critic) {
        hipLaunchKernelGGL(k_ds_train_bwd<1>, dim3(DSW_GRID), dim3(DSB_BLOCK), 0, s, p);
        if (int r = check_launch()) return r;
    }
    static_assert(DSW_SLOTS % (2 * DSR_GROUPS) == 0, "reduction stride");
    if (set_grads_out) {
        SetGradParams sg;
        const int nj = set_grad_params(setvec, dlogits, dmean, num_envs, num_elements, set_grads_out, sg);
        hipLaunchKernelGGL(k_ds_wgrad_reduce_sets, dim3(DSR_BLOCKS + SG_TILES * nj), dim3(SG_THREADS), 0, s, workspace,
                           wgrad_out, (int)actor, (int)critic, sg);
        return check_launch();
    }
    hipLaunchKernelGGL(k_ds_wgrad_reduce, dim3(DSR_BLOCKS), dim3(DSR_COLS * DSR_GROUPS), 0, s, workspace, wgrad_out,
                       (int)actor, (int)critic);
    return check_launch();
}
}  // namespace
extern "C" {

int lb_ds_train_backward(const float* bwd_frag, const float* obs, int64_t num_envs, int32_t num_elements,
                         const float* save_actor, const float* save_critic, const float* dlogits, const float* dmean,
                         float* wgrad_out, float* workspace, float* setvec, void* stream) {
    return train_backward(bwd_frag, obs, num_envs, num_elements, save_actor, save_critic, dlogits, dmean, wgrad_out,
                          workspace, setvec, nullptr, stream);
}

int lb_ds_train_backward_sets(const float* bwd_frag, const float* obs, int64_t num_envs, int32_t num_elements,
                              const float* save_actor, const float* save_critic, const float* dlogits,
                              const float* dmean, float* wgrad_out, float* workspace, float* setvec,
                              float* set_grads_out, void* stream) {
    if (!set_grads_out || !dlogits) return fail("lb_ds_train_backward_sets: set_grads_out and dlogits are required");
    return train_backward(bwd_frag, obs, num_envs, num_elements, save_actor, save_critic, dlogits, dmean, wgrad_out,
                          workspace, setvec, set_grads_out, stream);
}

int lb_ds_over_sets(const lb_set_job* jobs, int32_t num_jobs, int64_t num_sets, float* workspace,
                    int64_t workspace_floats, void* stream) {
    if (!jobs || num_jobs < 1 || num_jobs > OS_JOBS || num_sets < 1 || !workspace)
        return fail("lb_ds_over_sets: jobs NULL, num_jobs not in [1, 16], num_sets < 1 or workspace NULL");
    OverSetsParams p{};
    int row = 0;
    auto vec_ok = [](const float* x, int64_t ld) { return ((uintptr_t)x & 15) == 0 && ld % 4 == 0; };
    for (int i = 0; i < num_jobs; ++i) {
        const lb_set_job& j = jobs[i];
        if (!j.b || !j.out || j.M < 1 || j.N < 1 || j.M > 64 || j.N > 64 || (!j.a && j.M != 1))
            return fail("lb_ds_over_sets: a job needs b and out, 1 <= M, N <= 64 (M == 1 when a is NULL)");
        p.job[i] = OverSetsJob{j.a, j.lda, j.b, j.ldb, j.M, j.N, j.scale, j.out, row,
                               (vec_ok(j.a, j.lda) ? 1 : 0) | (vec_ok(j.b, j.ldb) ? 2 : 0)};
        row += j.M * j.N;
    }
    p.njobs = num_jobs;
    p.row = row;
    p.S = num_sets;
    p.work = workspace;
    const int64_t spans = (num_sets + OS_SPAN - 1) / OS_SPAN;
    if (spans * row > workspace_floats) return fail("lb_ds_over_sets: workspace too small (spans x outputs)");
    if (spans > 65535) return fail("lb_ds_over_sets: num_sets too large");
    hipLaunchKernelGGL(k_ds_over_sets, dim3((unsigned)((num_jobs + 3) / 4), (unsigned)spans), dim3(256), 0,
                       (hipStream_t)stream, p);
    if (int r = check_launch()) return r;
    hipLaunchKernelGGL(k_ds_over_sets_reduce, dim3((unsigned)((row + 63) / 64)), dim3(64 * OS_RG), 0, (hipStream_t)stream, p,
                       (int)spans);
    return check_launch();
}

int lb_ds_set_grads(const float* setvec, const float* dlogits, const float* dmean, int64_t num_sets,
                    int32_t num_elements, float* out, void* stream) {
    if (!setvec || !dlogits || !out || num_sets < 1) return fail("setvec/dlogits/out NULL or num_sets < 1");
    if (num_elements < 1 || num_elements > LB_DS_MAX_ELEMENTS_TRAIN)
        return fail("num_elements must be in [1, 257] (LB_DS_MAX_ELEMENTS_TRAIN)");
    SetGradParams p;
    const int nj = set_grad_params(setvec, dlogits, dmean, num_sets, num_elements, out, p);
    hipLaunchKernelGGL(k_ds_set_grads, dim3(SG_TILES, nj), dim3(SG_THREADS), 0, (hipStream_t)stream, p);
    return check_launch();
}

}  // extern "C"
