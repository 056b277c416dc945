"""Per-step `info` dicts and per-episode CSV rows rebuilt from the device accumulators.

Reference: loadbalancer_k8s_env.py:439-470 (13-key info, every value
float("{:.2f}")), :472-510 (episode end, two save_to_csv rows) and
utils.py:99-127 (CSV schema).  The GPU keeps exact integer counters and EXACT
fixed-point sums of the float lists per env (lbk8s_common.h xsum_add); this module
turns one env's accumulator row (the `ep_stats` layout below) into the reference's dict.

Means: the reference uses statistics.mean, i.e. the exact rational sum of the list
divided by its length, rounded once to float64 (:451-454, :491-506).  The row carries
each float sum exactly (a rounded float64 plus its exact remainder, or for the updated
topology list an integer residual D, include/lbk8s.h), so the mean here is the same
correctly rounded quotient, and "{:.2f}" formats the same float64.
"""
from fractions import Fraction

import numpy as np

INFO_KEYS = ("reward_step", "action", "reward", "ep_block_prob", "ep_accepted_requests",
             "avg_endpoint_latency", "avg_topology_latency", "avg_cost",
             "avg_cpu_endpoint_selected", "ep_intra_zone_percentage",
             "ep_inter_zone_percentage", "gini", "executionTime")

CSV_FIELDS = ("episode", "reward", "ep_block_prob", "ep_accepted_requests", "avg_endpoint_latency",
              "avg_topology_latency", "avg_cost", "avg_cpu_endpoint_selected",
              "ep_intra_zone_percentage", "ep_inter_zone_percentage", "gini", "execution_time")

# ep_stats row layout (float64 x 16), shared with the C-ABI (include/lbk8s.h LB_ST_*)
ST_RETURN, ST_LENGTH, ST_ACC, ST_SUM_LAT, ST_SUM_TOPO, ST_SUM_TOPO_UPD, ST_SUM_COST, \
    ST_SUM_CPU, ST_INTRA, ST_INTER, ST_GINI, ST_EPISODE, ST_SUM_LAT_REM, ST_SUM_CPU_REM, \
    ST_SUM_TOPO_UPD_D = range(15)
ST_K = 16
FIX_17 = 7656119366529843  # fl(1.7) * 2^52: INCREASE_COST_PERCENTAGE (:67) at scale 2^-52


def r2(x):
    """float("{:.2f}".format(x)) — the reference's rounding of every info value."""
    return float("{:.2f}".format(x))


def exact_sums(st):
    """The exact sums (Fractions) of the episode's latency, topology, cost, cpu and updated
    topology lists from one ep_stats row."""
    intra, topo = int(st[ST_INTRA]), int(st[ST_SUM_TOPO])
    lat = Fraction(float(st[ST_SUM_LAT])) + Fraction(float(st[ST_SUM_LAT_REM]))
    cpu = Fraction(float(st[ST_SUM_CPU])) + Fraction(float(st[ST_SUM_CPU_REM]))
    upd = intra + Fraction(FIX_17 * (topo - intra) - int(st[ST_SUM_TOPO_UPD_D]), 1 << 52)
    return lat, Fraction(topo), Fraction(int(st[ST_SUM_COST])), cpu, upd


def _avgs(st):
    """statistics.mean of the five lists: float(exact sum / count), correctly rounded."""
    acc = int(st[ST_ACC])
    if acc == 0:  # all four lists empty -> 1 (:444-449)
        return 1.0, 1.0, 1.0, 1.0, 1.0
    return tuple(float(x / acc) for x in exact_sums(st))


def step_info(st, reward, action, execution_time=0.0):
    """The 13-key info of loadbalancer_k8s_env.py:456-470 from one ep_stats row."""
    step = st[ST_LENGTH]
    avg_l, avg_t, avg_c, avg_cpu, _ = _avgs(st)
    return {
        "reward_step": r2(reward),
        "action": r2(action),
        "reward": r2(st[ST_RETURN]),
        "ep_block_prob": r2(1 - st[ST_ACC] / step),
        "ep_accepted_requests": r2(st[ST_ACC]),
        "avg_endpoint_latency": r2(avg_l),
        "avg_topology_latency": r2(avg_t),
        "avg_cost": r2(avg_c),
        "avg_cpu_endpoint_selected": r2(avg_cpu),
        "ep_intra_zone_percentage": r2(st[ST_INTRA] / step),
        "ep_inter_zone_percentage": r2(st[ST_INTER] / step),
        "gini": r2(st[ST_GINI]),
        "executionTime": r2(execution_time),
    }


def csv_rows(st, episode, execution_time=0.0):
    """The two save_to_csv rows written at episode end (:488-510): results + no_cost_updated.

    The reference raises StatisticsError here for an all-reject episode (mean([]));
    the framework writes the per-step convention (averages = 1) instead.
    """
    step = st[ST_LENGTH]
    avg_l, avg_t, avg_c, avg_cpu, avg_tu = _avgs(st)
    common = [r2(st[ST_RETURN]), r2(1 - st[ST_ACC] / step), r2(st[ST_ACC]), r2(avg_l)]
    tail = [r2(avg_c), r2(avg_cpu), r2(st[ST_INTRA] / step), r2(st[ST_INTER] / step),
            r2(st[ST_GINI]), r2(execution_time)]
    res = [int(episode)] + common + [r2(avg_t)] + tail
    upd = [int(episode)] + common + [r2(avg_tu)] + tail
    return dict(zip(CSV_FIELDS, res)), dict(zip(CSV_FIELDS, upd))


def info_matrix(stats, rewards, actions):
    """The 12 numeric info keys (no executionTime) for many envs: (B, 12) float64, each value
    exactly the reference's float("{:.2f}") (step_info per row)."""
    stats = np.asarray(stats, np.float64)
    out = np.empty((stats.shape[0], 12), np.float64)
    for b in range(stats.shape[0]):
        info = step_info(stats[b], float(rewards[b]), int(actions[b]))
        out[b] = [info[k] for k in INFO_KEYS[:12]]
    return out
