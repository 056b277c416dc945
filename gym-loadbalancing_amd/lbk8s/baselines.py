"""Greedy heuristic policies of envs/baselines.py:6-35.

Host form (same signatures, any env exposing the attributes): feasible endpoints are the
True entries of action_mask[:-1]; the last mask entry is dropped whether or not it is
the reject action (so without rejection the last endpoint is never chosen, as in the
reference); ties go to the lowest index (numpy argmin/argmax); with no feasible
endpoint the last action index is returned.

Batched device form: LBVecEnv.policy("topo" | "zone_cpu" | "endpoint_cpu") — the same
rule evaluated by k_policy for every env at once (masks are always all True, :808-821).
"""
import numpy as np


def _pick(values, action_mask, largest):
    feasible = np.flatnonzero(np.asarray(action_mask)[:-1])
    if feasible.size == 0:
        return len(action_mask) - 1
    v = np.asarray(values)[feasible]
    return int(feasible[np.argmax(v) if largest else np.argmin(v)])


def topology_greedy_policy(env, action_mask):
    """Feasible endpoint with the lowest topology latency to the request (:6-13)."""
    return _pick(env.endpoint_topology_latency, action_mask, largest=False)


def zone_cpu_greedy_policy(env, action_mask):
    """Feasible endpoint whose zone has the largest cpu capacity (:16-24)."""
    return _pick(env.endpoint_zone_cpu_capacity, action_mask, largest=True)


def endpoint_cpu_greedy_policy(env, action_mask):
    """Feasible endpoint with the lowest cpu usage (:27-35)."""
    return _pick(env.endpoint_cpu_usage_percentage, action_mask, largest=False)


POLICIES = {"topo": topology_greedy_policy, "zone_cpu": zone_cpu_greedy_policy,
            "endpoint_cpu": endpoint_cpu_greedy_policy}
