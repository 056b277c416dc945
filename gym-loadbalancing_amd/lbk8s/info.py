"""Per-step `info` dicts and per-episode CSV rows rebuilt from the device accumulators.

Reference: loadbalancer_k8s_env.py:439-470 (13-key info, every value
float("{:.2f}")), :472-510 (episode end, two save_to_csv rows) and
utils.py:99-127 (CSV schema).  The GPU keeps exact integer counters and float64
running sums per env; this module turns one env's accumulator row (the
`ep_stats` layout below) into the reference's dict.

Means: the reference uses statistics.mean (exact rational) over per-episode
lists; here sum/count in float64.  For integer-valued lists (topology latency,
cost) that is bit-identical; for float lists the 2-decimal value differs only
when the exact mean lies within ~1e-13 of a rounding boundary.
"""
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
    ST_SUM_CPU, ST_INTRA, ST_INTER, ST_GINI, ST_EPISODE = range(12)
ST_K = 16


def r2(x):
    """float("{:.2f}".format(x)) — the reference's rounding of every info value."""
    return float("{:.2f}".format(x))


def _avgs(st):
    acc = st[ST_ACC]
    if acc == 0:  # all four lists empty -> 1 (:444-449)
        return 1.0, 1.0, 1.0, 1.0, 1.0
    return (st[ST_SUM_LAT] / acc, st[ST_SUM_TOPO] / acc, st[ST_SUM_COST] / acc,
            st[ST_SUM_CPU] / acc, st[ST_SUM_TOPO_UPD] / acc)


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
    """Vectorised 12 numeric info keys (no executionTime) for many envs: (B, 12) float64."""
    stats = np.asarray(stats, np.float64)
    acc = stats[:, ST_ACC]
    step = np.maximum(stats[:, ST_LENGTH], 1)
    safe = np.where(acc > 0, acc, 1)
    avg = lambda k: np.where(acc > 0, stats[:, k] / safe, 1.0)  # noqa: E731
    cols = [rewards, actions, stats[:, ST_RETURN], 1 - acc / step, acc, avg(ST_SUM_LAT),
            avg(ST_SUM_TOPO), avg(ST_SUM_COST), avg(ST_SUM_CPU), stats[:, ST_INTRA] / step,
            stats[:, ST_INTER] / step, stats[:, ST_GINI]]
    return np.round(np.stack([np.asarray(c, np.float64) for c in cols], axis=1), 2)
