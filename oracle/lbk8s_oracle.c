/*
 * lbk8s_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A plain-C, CPU restatement of the reference LoadBalancerK8sEnv hot path
 * (/root/reference/envs/loadbalancer_k8s_env.py, envs/utils.py, envs/baselines.py),
 * batched over B independent envs.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  It deliberately keeps the
 * reference's DIRECT state representation (float64 endpoint latency / CPU
 * arrays, per-node CPU, the "heap" as a pending-endpoint slot, stale
 * selected_* values) so that it is an independent check of the GPU kernel,
 * which uses a compressed history-count representation.
 *
 * Parity pin: tests/test_oracle_golden.py checks this file against the golden
 * fixtures produced by running the reference itself (tests/golden/gen_golden.py).
 *
 * Draw sources:
 *   - trace  : RNG values injected per call (the numpy draws the reference made);
 *   - philox : the framework's own counter-based stream, restated
 *              here independently of the device code so both must agree bit-for-bit.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp). No FMA
 * contraction anywhere: the reference's float64 arithmetic is plain IEEE mul/div.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- constants (loadbalancer_k8s_env.py:17-79, utils.py:33-64) ---------- */
static const double NODE_CPU[5] = {2.0, 2.0, 2.0, 4.0, 8.0};   /* :35-39 'cpu'  */
static const int NODE_COST[5] = {1, 2, 4, 8, 16};              /* :35-39 'cost' */
static const int THRESHOLDS[7] = {400, 200, 150, 250, 450, 375, 500}; /* utils.py:33-64 */
#define DEFAULT_NUM_ZONES 4   /* :46, hard-coded zone draw range (:205,:354) */
#define DEFAULT_NUM_NODES 24  /* :47, hard-coded endpoint host range (:242,:380) */
#define INCREASE_COST_PERCENTAGE 1.7 /* :67 */

enum { RF_NAIVE = 0, RF_LATENCY = 1, RF_FAIRNESS = 2, RF_MULTI = 3 };

typedef struct {
    int32_t num_endpoints, num_zones, num_nodes, episode_length;
    int32_t reward_fn, rejection_allowed, auto_reset, rng_mode; /* rng_mode 0 philox, 1 trace */
    double arrival_rate, call_duration, latency_weight, cpu_weight, gini_weight;
    uint64_t seed;
    int64_t env_id_offset;
} orc_cfg;

typedef struct {
    const double *x1, *x2;
    const int32_t *r, *n;
} orc_step_trace;

typedef struct {
    const double *lat0;                     /* [B*E] */
    const int32_t *topo;                    /* [B*Z*(Z-1)], loop order of :331-338 */
    const int32_t *ntype, *nzone, *ncpu;    /* [B*N] */
    const int32_t *enode;                   /* [B*E] */
    const double *x1, *x2;                  /* [B] request draws closing reset() */
    const int32_t *r, *n;
} orc_reset_trace;

typedef struct {
    orc_cfg c;
    int64_t B;
    int E, Z, N, R;
    /* endpoint arrays [B*E] */
    int32_t *ep_node, *ep_zone;
    double *ep_cap, *ep_cpu, *ep_lat, *ep_topo, *loads;
    /* node arrays [B*N] */
    int32_t *node_type, *node_zone;
    double *node_cpu;
    /* zone arrays */
    double *zone_cap; /* [B*Z] */
    double *topo;     /* [B*Z*Z] */
    /* per-env scalars [B] */
    double *t, *dt, *sel_lat, *sel_topo, *sel_cpu, *total_reward;
    double *last_rw;  /* the float64 reward of the last step (get_reward() :516-567) */
    unsigned __int128 *sum_lat, *sum_topo_upd, *sum_cpu;  /* exact sums of the lists, x 2^52 */
    int64_t *sum_topo, *sum_cost;
    int32_t *step, *acc, *intra, *inter, *penalty, *pending, *req_zone, *req_thr, *req_node;
    uint32_t *episode;
    int32_t *was_reset;
} orc_env;

/* ---------------- Philox4x32-R (Salmon et al., SC'11) -------------------- */
/* The draw map runs ORC_PHILOX_ROUNDS = 10 (Philox4x32-10, the Random123 default);
 * orc_philox_r exposes the round count so tests pin it against the Random123
 * philox4x32_10 known answers. */
#define ORC_PHILOX_ROUNDS 10
static void philox4x32_r(uint32_t ctr[4], uint32_t k0, uint32_t k1, int rounds, uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    for (int i = 0; i < rounds; ++i) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* domains of the framework's draw map */
enum { D_INIT = 1, D_NODE = 2, D_EP = 3, D_TOPO = 4, D_REQ_X = 5, D_REQ_I = 6, D_ACT = 7, D_DQN_EXPLORE = 8,
       D_DQN_SAMPLE = 9 };

static void draw(const orc_env* s, int64_t b, uint32_t episode, uint32_t slot, uint32_t dom,
                 uint32_t out[4]) {
    uint64_t gid = (uint64_t)(s->c.env_id_offset + b);
    uint32_t ctr[4] = {(uint32_t)gid, episode, slot, dom | ((uint32_t)(gid >> 32) << 8)};
    philox4x32_r(ctr, (uint32_t)s->c.seed, (uint32_t)(s->c.seed >> 32), ORC_PHILOX_ROUNDS, out);
}

static uint32_t bounded(uint32_t w, uint32_t n) { return (uint32_t)(((uint64_t)w * n) >> 32); }
static double u53(uint32_t hi, uint32_t lo) {
    uint64_t x = (((uint64_t)hi << 32) | lo) >> 11;
    return (double)x * (1.0 / 9007199254740992.0);
}

/* log(x) for x in (0,1]: the fdlibm e_log.c reduction + minimax polynomial,
 * written out with plain IEEE ops so host and device agree bit-for-bit. */
static double fd_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    uint64_t bits;
    memcpy(&bits, &x, 8);
    int k = (int)((bits >> 52) & 0x7ff) - 1023;
    uint64_t mb = (bits & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL;
    double m;
    memcpy(&m, &mb, 8);
    if (m > 1.4142135623730951) { m = m * 0.5; k += 1; }
    double f = m - 1.0;
    double sv = f / (2.0 + f);
    double z = sv * sv, w = z * z;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    double Rr = t2 + t1;
    double hfsq = 0.5 * f * f;
    double dk = (double)k;
    return dk * ln2_hi - ((hfsq - (sv * (hfsq + Rr) + dk * ln2_lo)) - f);
}
static double std_exp(uint32_t hi, uint32_t lo) { return -fd_log(1.0 - u53(hi, lo)); }

/* ---------------- exact list sums (statistics.mean, :451-454) ------------- */
/* Every value appended to the reference's float lists is a float64 in [1, 1024), so
 * x * 2^52 is an integer below 2^62 and the list's exact sum is an integer at scale 2^-52
 * (unsigned __int128 here).  The device keeps the same sums as 64-bit words plus packed
 * carries (lbk8s_common.h xsum_add); both hand out the same ep_stats columns. */
static unsigned __int128 fix52(double x) { return (unsigned __int128)(uint64_t)ldexp(x, 52); }
/* the correctly rounded sum and its exact remainder (LB_ST_SUM_* / LB_ST_SUM_*_REM) */
static void fix_pair(unsigned __int128 v, double* s, double* r) {
    uint64_t hi = (uint64_t)(v >> 64), lo = (uint64_t)v;
    double xh = ldexp((double)hi, 64) + ldexp((double)(uint32_t)(lo >> 32), 32);
    double xl = (double)(uint32_t)lo;
    double sum = xh + xl;
    *s = ldexp(sum, -52);
    *r = ldexp(xl - (sum - xh), -52);
}
#define FIX_17 7656119366529843ULL  /* fl(1.7) * 2^52 */

/* ---------------- lifecycle ---------------------------------------------- */
#define ALLOC(p, n) ((p) = calloc((size_t)(n), sizeof(*(p))))

void* orc_create(const orc_cfg* cfg, int64_t B) {
    orc_env* s = calloc(1, sizeof(orc_env));
    s->c = *cfg;
    s->B = B;
    s->E = cfg->num_endpoints; s->Z = cfg->num_zones; s->N = cfg->num_nodes;
    s->R = s->E + (cfg->rejection_allowed ? 1 : 0);
    int64_t BE = B * s->E, BN = B * s->N;
    ALLOC(s->ep_node, BE); ALLOC(s->ep_zone, BE); ALLOC(s->ep_cap, BE); ALLOC(s->ep_cpu, BE);
    ALLOC(s->ep_lat, BE); ALLOC(s->ep_topo, BE); ALLOC(s->loads, BE);
    ALLOC(s->node_type, BN); ALLOC(s->node_zone, BN); ALLOC(s->node_cpu, BN);
    ALLOC(s->zone_cap, B * s->Z); ALLOC(s->topo, B * s->Z * s->Z);
    ALLOC(s->t, B); ALLOC(s->dt, B); ALLOC(s->sel_lat, B); ALLOC(s->sel_topo, B); ALLOC(s->sel_cpu, B);
    ALLOC(s->total_reward, B); ALLOC(s->last_rw, B); ALLOC(s->sum_lat, B); ALLOC(s->sum_topo_upd, B); ALLOC(s->sum_cpu, B);
    ALLOC(s->sum_topo, B); ALLOC(s->sum_cost, B);
    ALLOC(s->step, B); ALLOC(s->acc, B); ALLOC(s->intra, B); ALLOC(s->inter, B); ALLOC(s->penalty, B);
    ALLOC(s->pending, B); ALLOC(s->req_zone, B); ALLOC(s->req_thr, B); ALLOC(s->req_node, B);
    ALLOC(s->episode, B); ALLOC(s->was_reset, B);
    for (int64_t b = 0; b < B; ++b) s->pending[b] = -1;
    return s;
}

void orc_destroy(void* h) {
    orc_env* s = h;
    void* ptrs[] = {s->ep_node, s->ep_zone, s->ep_cap, s->ep_cpu, s->ep_lat, s->ep_topo, s->loads,
                    s->node_type, s->node_zone, s->node_cpu, s->zone_cap, s->topo, s->t, s->dt,
                    s->sel_lat, s->sel_topo, s->sel_cpu, s->total_reward, s->last_rw, s->sum_lat,
                    s->sum_topo_upd, s->sum_cpu, s->sum_topo, s->sum_cost, s->step, s->acc,
                    s->intra, s->inter, s->penalty, s->pending, s->req_zone, s->req_thr,
                    s->req_node, s->episode, s->was_reset};
    for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); ++i) free(ptrs[i]);
    free(s);
}

static double clamp_cpu(double v) { double m = v < 100.0 ? v : 100.0; return m > 1.0 ? m : 1.0; }
static double clamp_lat(double v) { double m = v < 500.0 ? v : 500.0; return m > 1.0 ? m : 1.0; }

/* next_request() :1131-1163 incl. dequeue_request :1090-1105 and deployment_generator :1114-1128 */
static void next_request(orc_env* s, int64_t b, double x1, double x2, int r, int n) {
    int E = s->E;
    double arrival = s->t[b] + x1;
    double departure = arrival + x2;
    s->dt[b] = departure - arrival;
    s->t[b] = arrival;
    int e = s->pending[b];        /* heap holds <=1 request with departure_time 0 < arrival */
    if (e >= 0) {
        int h = s->ep_node[b * E + e];
        double* nc = &s->node_cpu[b * s->N + h];
        *nc = clamp_cpu(*nc / 1.15);                       /* decrease_resources :937-960 */
        s->ep_cpu[b * E + e] = *nc;
        double prev = trunc(s->ep_lat[b * E + e]);         /* decrease_endpoint_latency :1052-1060 */
        s->ep_lat[b * E + e] = clamp_lat(prev / 1.15);
        s->pending[b] = -1;
    }
    int idx = r - 1;                                      /* endpoint_list[random - 1] :1117 */
    if (idx < 0) idx += 7;
    s->req_thr[b] = THRESHOLDS[idx];
    s->req_node[b] = n;
    s->req_zone[b] = s->node_zone[b * s->N + n];
    for (int k = 0; k < E; ++k)                           /* :1161-1163 */
        s->ep_topo[b * E + k] = s->topo[(b * s->Z + s->ep_zone[b * E + k]) * s->Z + s->req_zone[b]];
}

static void write_obs(const orc_env* s, int64_t b, float* obs) {
    int E = s->E;
    float* o = obs + b * (int64_t)s->R * 8;
    for (int k = 0; k < E; ++k) {
        float* row = o + k * 8;
        row[0] = (float)s->ep_zone[b * E + k];
        row[1] = (float)s->ep_cap[b * E + k];
        row[2] = (float)s->ep_cpu[b * E + k];
        row[3] = (float)s->ep_topo[b * E + k];
        row[4] = (float)s->ep_lat[b * E + k];
        row[5] = (float)s->req_zone[b];
        row[6] = (float)s->req_thr[b];
        row[7] = (float)s->dt[b];
    }
    if (s->c.rejection_allowed) {
        float* row = o + E * 8;
        for (int j = 0; j < 5; ++j) row[j] = -1.0f;
        row[5] = (float)s->req_zone[b];
        row[6] = (float)s->req_thr[b];
        row[7] = (float)s->dt[b];
    }
}

/* reset() :290-400 for one env */
static void reset_one(orc_env* s, int64_t b, const orc_reset_trace* tr) {
    int E = s->E, Z = s->Z, N = s->N;
    s->step[b] = 0; s->total_reward[b] = 0.0; s->acc[b] = 0; s->penalty[b] = 0;
    s->intra[b] = 0; s->inter[b] = 0;
    s->sum_lat[b] = 0; s->sum_topo_upd[b] = 0; s->sum_cpu[b] = 0;
    s->sum_topo[b] = 0; s->sum_cost[b] = 0;
    s->sel_lat[b] = 0.0; s->sel_topo[b] = 0.0; s->sel_cpu[b] = 1.0;   /* :325-327 */
    s->episode[b] += 1;
    uint32_t ep = s->episode[b];
    uint32_t w[4];
    for (int k = 0; k < E; ++k) s->loads[b * E + k] = 0.0;
    /* latency ~ U(1,100) :328 */
    for (int k = 0; k < E; ++k) {
        double v;
        if (tr) v = tr->lat0[b * E + k];
        else { draw(s, b, ep, (uint32_t)k, D_EP, w); v = 1.0 + 99.0 * u53(w[0], w[1]); }
        s->ep_lat[b * E + k] = v;
    }
    /* topology :331-338 — symmetric, diag 1, last writer wins */
    double* T = s->topo + b * Z * Z;
    if (tr) {
        const int32_t* d = tr->topo + b * Z * (Z - 1);
        int k = 0;
        for (int z1 = 0; z1 < Z; ++z1)
            for (int z2 = 0; z2 < Z; ++z2) {
                if (z1 == z2) T[z1 * Z + z2] = 1.0;
                else { T[z1 * Z + z2] = d[k]; T[z2 * Z + z1] = d[k]; ++k; }
            }
    } else {
        for (int i = 0; i < Z * Z; ++i) T[i] = 0.0;
        for (int z = 0; z < Z; ++z) T[z * Z + z] = 1.0;
        uint32_t w2[4];
        draw(s, b, ep, 0, D_TOPO, w);
        draw(s, b, ep, 1, D_TOPO, w2);
        uint32_t words[6] = {w[0], w[1], w[2], w[3], w2[0], w2[1]};
        int p = 0;
        for (int i = 0; i < DEFAULT_NUM_ZONES; ++i)
            for (int j = i + 1; j < DEFAULT_NUM_ZONES; ++j) {
                double v = 1.0 + bounded(words[p++], 499);
                T[i * Z + j] = v; T[j * Z + i] = v;
            }
    }
    /* nodes :344-362 and node cpu :369-373 */
    double* zc = s->zone_cap + b * Z;
    for (int z = 0; z < Z; ++z) zc[z] = 0.0;
    for (int n = 0; n < N; ++n) {
        int ty, zo, cpu;
        if (tr) { ty = tr->ntype[b * N + n]; zo = tr->nzone[b * N + n]; cpu = tr->ncpu[b * N + n]; }
        else {
            draw(s, b, ep, (uint32_t)n, D_NODE, w);
            ty = (int)bounded(w[0], 5); zo = (int)bounded(w[1], DEFAULT_NUM_ZONES);
            cpu = 1 + (int)bounded(w[2], 99);
        }
        s->node_type[b * N + n] = ty;
        s->node_zone[b * N + n] = zo;
        zc[zo] += NODE_CPU[ty];
        s->node_cpu[b * N + n] = (double)cpu;
    }
    /* endpoints :379-386 */
    for (int k = 0; k < E; ++k) {
        int node;
        if (tr) node = tr->enode[b * E + k];
        else { draw(s, b, ep, (uint32_t)k, D_EP, w); node = (int)bounded(w[2], DEFAULT_NUM_NODES); }
        s->ep_node[b * E + k] = node;
        s->ep_zone[b * E + k] = s->node_zone[b * N + node];
        s->ep_cpu[b * E + k] = s->node_cpu[b * N + node];
        s->ep_cap[b * E + k] = zc[s->node_zone[b * N + node]];
    }
    s->penalty[b] = 0;
    /* next_request() :397 */
    double x1, x2;
    int r, n;
    if (tr) { x1 = tr->x1[b]; x2 = tr->x2[b]; r = tr->r[b]; n = tr->n[b]; }
    else {
        uint32_t wi[4];
        draw(s, b, ep, 0, D_REQ_X, w);
        draw(s, b, ep, 0, D_REQ_I, wi);
        x1 = (1.0 / s->c.arrival_rate) * std_exp(w[0], w[1]);
        x2 = s->c.call_duration * std_exp(w[2], w[3]);
        r = (int)bounded(wi[0], 7); n = (int)bounded(wi[1], (uint32_t)N);
    }
    next_request(s, b, x1, x2, r, n);
}

/* __init__: the only state that survives into reset() is current_time. */
void orc_init(void* h, const double* t0) {
    orc_env* s = h;
    for (int64_t b = 0; b < s->B; ++b) {
        s->episode[b] = 0;
        if (t0) s->t[b] = t0[b];
        else {
            uint32_t w[4];
            draw(s, b, 0, 0, D_INIT, w);
            s->t[b] = 0.0 + (1.0 / s->c.arrival_rate) * std_exp(w[0], w[1]);
        }
    }
}

void orc_reset(void* h, const uint8_t* mask, float* obs, const orc_reset_trace* tr) {
    orc_env* s = h;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < s->B; ++b) {
        if (mask && !mask[b]) continue;
        reset_one(s, b, tr);
        if (obs) write_obs(s, b, obs);
    }
}

static double gini(const orc_env* s, int64_t b) {   /* utils.py:132-143 */
    int n = s->E;
    const double* l = s->loads + b * n;
    double total = 0.0;
    for (int i = 0; i < n; ++i) total += l[i];
    double mean = total / n;
    if (mean == 0.0) return 0.0;
    double num = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) num += fabs(l[i] - l[j]);
    return num / ((double)(2 * n * n) * mean);
}

/* get_reward() :516-567 */
static double reward_of(const orc_env* s, int64_t b) {
    switch (s->c.reward_fn) {
    case RF_NAIVE: return s->penalty[b] ? -1.0 : 1.0;
    case RF_LATENCY: return s->penalty[b] ? -1000.0 : -(s->sel_lat[b] + s->sel_topo[b]);
    case RF_FAIRNESS: return s->penalty[b] ? -1.0 : 1.0 - gini(s, b);
    default: {
        if (s->penalty[b]) return -1.0;
        double current = s->sel_lat[b] + s->sel_topo[b];
        double cpu = s->sel_cpu[b];
        double g = gini(s, b);
        current = (current - 2.0) / (1000.0 - 2.0);            /* utils.normalize */
        cpu = (cpu - 1.0) / (100.0 - 1.0);
        return s->c.latency_weight * (1.0 - current) + s->c.cpu_weight * (1.0 - cpu) +
               s->c.gini_weight * (1.0 - g);
    }
    }
}

enum { ST_RETURN, ST_LENGTH, ST_ACC, ST_SUM_LAT, ST_SUM_TOPO, ST_SUM_TOPO_UPD, ST_SUM_COST,
       ST_SUM_CPU, ST_INTRA, ST_INTER, ST_GINI, ST_EPISODE, ST_SUM_LAT_REM, ST_SUM_CPU_REM,
       ST_SUM_TOPO_UPD_D, ST_K = 16 };

static void stats_of(const orc_env* s, int64_t b, double* st) {
    st[ST_RETURN] = s->total_reward[b];
    st[ST_LENGTH] = s->step[b];
    st[ST_ACC] = s->acc[b];
    fix_pair(s->sum_lat[b], &st[ST_SUM_LAT], &st[ST_SUM_LAT_REM]);
    st[ST_SUM_TOPO] = (double)s->sum_topo[b];
    /* float64 approximation (as the device writes it); the exact sum via D below */
    st[ST_SUM_TOPO_UPD] = (double)s->intra[b] + 1.7 * (double)(s->sum_topo[b] - s->intra[b]);
    st[ST_SUM_COST] = (double)s->sum_cost[b];
    fix_pair(s->sum_cpu[b], &st[ST_SUM_CPU], &st[ST_SUM_CPU_REM]);
    st[ST_INTRA] = s->intra[b];
    st[ST_INTER] = s->inter[b];
    st[ST_GINI] = gini(s, b);
    st[ST_EPISODE] = s->episode[b];
    /* D = intra * 2^52 + M * (sum_topo - intra) - exact updated sum (include/lbk8s.h) */
    unsigned __int128 m = (unsigned __int128)s->intra[b] << 52;
    m += (unsigned __int128)FIX_17 * (uint64_t)(s->sum_topo[b] - s->intra[b]);
    st[ST_SUM_TOPO_UPD_D] = (double)(__int128)(m - s->sum_topo_upd[b]);
    st[ST_K - 1] = 0.0;
}

/* step() :403-513 (+ VecEnv auto-reset when cfg.auto_reset) */
void orc_step(void* h, const int32_t* actions, float* obs, float* reward, uint8_t* done,
              float* terminal_obs, double* ep_stats, const orc_step_trace* st_tr,
              const orc_reset_trace* rs_tr) {
    orc_env* s = h;
    int E = s->E, Z = s->Z;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < s->B; ++b) {
        int a = actions[b];
        /* take_action :578-686 */
        s->step[b] += 1;
        if (a < -E) {
            /* the reference raises IndexError here; the framework treats it like an
             * unrecognised action (penalty stale) and flags it */
        } else if (a < E) {
            int ai = a < 0 ? a + E : a;                 /* Python negative indexing */
            int64_t i = b * E + ai;
            s->acc[b] += 1;
            int in_zone = s->req_zone[b];
            int out_zone = s->ep_zone[i];
            int h = s->ep_node[i];
            int cost = NODE_COST[s->node_type[b * s->N + h]];
            double tl = s->topo[(b * Z + in_zone) * Z + out_zone];
            double tu = in_zone == out_zone ? 1.0 : s->topo[(b * Z + in_zone) * Z + out_zone] *
                                                       INCREASE_COST_PERCENTAGE;
            s->sum_topo[b] += (int64_t)tl;
            s->sum_topo_upd[b] += fix52(tu);
            s->sum_lat[b] += fix52(s->ep_lat[i]);
            s->sum_cost[b] += cost;
            s->loads[i] += 1.0;
            s->sum_cpu[b] += fix52(s->ep_cpu[i]);
            s->sel_lat[b] = s->ep_lat[i];
            s->sel_topo[b] = tl;
            s->sel_cpu[b] = s->ep_cpu[i];
            if (in_zone == out_zone) s->intra[b] += 1; else s->inter[b] += 1;
            s->pending[b] = ai;                          /* enqueue_request :671 */
            double* nc = &s->node_cpu[b * s->N + h];    /* increase_resources :861-887 */
            *nc = clamp_cpu(*nc * 1.15);
            s->ep_cpu[i] = *nc;
            double prev = trunc(s->ep_lat[i]);          /* increase_endpoint_latency :1013-1023 */
            s->ep_lat[i] = clamp_lat(prev * 1.5);
            s->penalty[b] = 0;
        } else if (a == E) {
            s->penalty[b] = 1;
        } /* else: unrecognised action, penalty stale (:685-686) */
        double rw = reward_of(s, b);
        s->total_reward[b] += rw;
        s->last_rw[b] = rw;
        double x1, x2;
        int r, n;
        if (st_tr) { x1 = st_tr->x1[b]; x2 = st_tr->x2[b]; r = st_tr->r[b]; n = st_tr->n[b]; }
        else {
            uint32_t w[4], wi[4];
            draw(s, b, s->episode[b], (uint32_t)s->step[b], D_REQ_X, w);
            draw(s, b, s->episode[b], (uint32_t)s->step[b], D_REQ_I, wi);
            x1 = (1.0 / s->c.arrival_rate) * std_exp(w[0], w[1]);
            x2 = s->c.call_duration * std_exp(w[2], w[3]);
            r = (int)bounded(wi[0], 7); n = (int)bounded(wi[1], (uint32_t)s->N);
        }
        next_request(s, b, x1, x2, r, n);
        int d = s->step[b] == s->c.episode_length;
        if (reward) reward[b] = (float)rw;
        if (done) done[b] = (uint8_t)d;
        if (d && ep_stats) stats_of(s, b, ep_stats + b * ST_K);
        if (d && s->c.auto_reset) {
            if (terminal_obs) write_obs(s, b, terminal_obs);
            reset_one(s, b, rs_tr);
        }
        if (obs) write_obs(s, b, obs);
    }
}

/* the float64 rewards of the last orc_step (what the reference's step() returns, :513, before
 * SubprocVecEnv / VecMonitor see it: run.py:114-122) */
void orc_last_reward64(void* h, double* out) {
    orc_env* s = h;
    for (int64_t b = 0; b < s->B; ++b) out[b] = s->last_rw[b];
}

void orc_get_stats(void* h, double* out) {
    orc_env* s = h;
    for (int64_t b = 0; b < s->B; ++b) stats_of(s, b, out + b * ST_K);
}

/* baselines.py:6-35 — greedy argmin/argmax over feasible = mask[:-1] (all True). */
void orc_policy_greedy(void* h, int kind, int32_t* actions) {
    orc_env* s = h;
    int E = s->E;
    int A = s->c.rejection_allowed ? E + 1 : E;
    int nf = A - 1;
    for (int64_t b = 0; b < s->B; ++b) {
        if (nf <= 0) { actions[b] = A - 1; continue; }
        const double* v = kind == 0 ? s->ep_topo + b * E : kind == 1 ? s->ep_cap + b * E : s->ep_cpu + b * E;
        int best = 0;
        for (int k = 1; k < nf; ++k) {
            if (kind == 1 ? v[k] > v[best] : v[k] < v[best]) best = k;
        }
        actions[b] = best;
    }
}

/* random policy (bench / Philox mode): a ~ U{0..A-1}, keyed by (env, episode, step). */
void orc_policy_random(void* h, int32_t* actions) {
    orc_env* s = h;
    int A = s->c.rejection_allowed ? s->E + 1 : s->E;
    for (int64_t b = 0; b < s->B; ++b) {
        uint32_t w[4];
        draw(s, b, s->episode[b], (uint32_t)s->step[b], D_ACT, w);
        actions[b] = (int32_t)bounded(w[0], (uint32_t)A);
    }
}

/* state views for tests: field ids mirror lb_get_field in include/lbk8s.h */
void orc_get_field(void* h, int field, double* out) {
    orc_env* s = h;
    int64_t BE = s->B * s->E;
    switch (field) {
    case 0: for (int64_t i = 0; i < BE; ++i) out[i] = s->ep_lat[i]; break;
    case 1: for (int64_t i = 0; i < BE; ++i) out[i] = s->ep_cpu[i]; break;
    case 2: for (int64_t i = 0; i < BE; ++i) out[i] = s->ep_topo[i]; break;
    case 3: for (int64_t i = 0; i < BE; ++i) out[i] = s->ep_cap[i]; break;
    case 4: for (int64_t i = 0; i < BE; ++i) out[i] = s->ep_zone[i]; break;
    case 5: for (int64_t i = 0; i < BE; ++i) out[i] = s->ep_node[i]; break;
    case 6: for (int64_t i = 0; i < BE; ++i) out[i] = s->loads[i]; break;
    case 7: for (int64_t b = 0; b < s->B; ++b) out[b] = s->t[b]; break;
    case 8: for (int64_t b = 0; b < s->B; ++b) out[b] = s->step[b]; break;
    case 9: for (int64_t b = 0; b < s->B; ++b) out[b] = s->req_zone[b]; break;
    case 10: for (int64_t b = 0; b < s->B; ++b) out[b] = s->req_thr[b]; break;
    case 11: for (int64_t b = 0; b < s->B; ++b) out[b] = s->dt[b]; break;
    case 12: for (int64_t i = 0; i < s->B * s->N; ++i) out[i] = s->node_cpu[i]; break;
    default: break;
    }
}

int orc_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* expose the RNG primitives so tests can pin them against known-answer vectors */
void orc_philox_r(const uint32_t ctr[4], uint32_t k0, uint32_t k1, int32_t rounds,
                  uint32_t out[4]) {
    uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
    philox4x32_r(c, k0, k1, rounds, out);
}
int32_t orc_philox_rounds(void) { return ORC_PHILOX_ROUNDS; }
double orc_log(double x) { return fd_log(x); }

/* The DQN's device decisions (include/lbk8s.h lb_dqn_act, lb_replay_sample), restated:
 * dqn_deepset.py:125-127's epsilon-greedy draw at vector step t -- eps = linear_schedule
 * (:32-34) = max(slope t + start_e, end_e), one u53 keyed by (seed, t) -- and SB3
 * ReplayBuffer.sample's (slot, env) of sample i drawn at counter t. */
int32_t orc_dqn_explore(uint64_t seed, double start_e, double slope, double end_e, int64_t t) {
    const double a = slope * (double)t + start_e;
    const double eps = a > end_e ? a : end_e;
    uint32_t ctr[4] = {(uint32_t)t, (uint32_t)((uint64_t)t >> 32), 0u, D_DQN_EXPLORE}, w[4];
    philox4x32_r(ctr, (uint32_t)seed, (uint32_t)(seed >> 32), ORC_PHILOX_ROUNDS, w);
    return u53(w[0], w[1]) < eps ? 1 : 0;
}
void orc_replay_sample(uint64_t seed, int64_t t, int64_t upper, int64_t n_envs, int32_t batch, int64_t* slot,
                       int64_t* env) {
    for (int32_t i = 0; i < batch; ++i) {
        uint32_t ctr[4] = {(uint32_t)t, (uint32_t)((uint64_t)t >> 32), (uint32_t)i, D_DQN_SAMPLE}, w[4];
        philox4x32_r(ctr, (uint32_t)seed, (uint32_t)(seed >> 32), ORC_PHILOX_ROUNDS, w);
        slot[i] = (int64_t)(((uint64_t)w[0] * (uint64_t)upper) >> 32);
        env[i] = (int64_t)bounded(w[1], (uint32_t)n_envs);
    }
}

/* Re-key the Philox stream (LBVecEnv.seed(): applied at the next full reset). */
void orc_set_seed(void* h, uint64_t seed) { ((orc_env*)h)->c.seed = seed; }
