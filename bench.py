#!/usr/bin/env python3
"""Benchmark: vectorized LoadBalancerK8sEnv env-steps/s on MI355X (BASELINE.json config 3).

One bench "step" = one vector step of every env on every GPU: take_action + reward +
next_request + get_state + auto-reset with the env's uniform random policy drawn on the
device (the random policy of BASELINE configs 2/3, the same draws lb_policy(random)
returns).  Observations, rewards and dones go into a T-deep device ring, the shape of PPO's
rollout storage (ppo_deepset.py:136-143; T = 100 as SURVEY 8d sizes it), so writes stream to
HBM instead of sitting in the 256 MB Infinity Cache; terminal observations and episode-statistics rows of finished envs
are written too.  Env state is resident in HBM before timing.

Two launch shapes run the same steps (bit for bit, tests/test_gpu_api.py):
  --launch rollout (default): lb_rollout, K = T = 100 vector steps per launch (k_rollout_lean),
      the env state in registers between the steps of a launch, every step's outputs in
      its ring slot -- the step-only workload of config 3 (no host policy in the loop);
  --launch step: one lb_step launch per vector step (k_step_tpe), the VecEnv.step() shape
      a host/NN policy needs; measured in the same run and reported under "lb_step".

Episodes are staggered before timing (env i starts at step i mod episode_length), so every
timed step ends and auto-resets 1/episode_length of the envs — the steady state of a
long-running VecEnv — whatever --steps is; the count of resets inside the timed window is
reported.

Default workload: 2^20 default-scenario envs IN TOTAL (E=8, N=24, Z=4, rejection, naive,
episode_length 100; Philox seed 0), sharded over the GPUs: rank r owns global env ids
[r*B/G, (r+1)*B/G) with no data-path collective ("scaling": "strong").  --weak keeps
--envs per GPU instead.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  With --gpus N > 1 and no torchrun environment, bench.py launches N ranks itself
  (torch.distributed.run, 127.0.0.1) before touching the GPU and exits with their status.
  --plan-only: the launcher / sharding / statistics-reduction path without a GPU (gloo).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "gym-loadbalancing_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "env-steps/sec (whole node) at 1M envs, 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
REFERENCE_SUBPROC_8CORE = 2858.0  # the reference itself, 8-worker pipe VecEnv, survey container

CONFIGS = {
    "default": dict(),  # constructor defaults, loadbalancer_k8s_env.py:42-54
    "cfg1": dict(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="naive",
                 latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0),
    "e64_multi": dict(num_endpoints=64, reward_function="multi", latency_weight=1.0,
                      cpu_weight=0.0, gini_weight=0.0),
}


def algorithmic_bytes(cfg, reads_actions=True):
    """B_alg = 53*E + 6*Z + 240 (rejection) / + 208 (no rejection), which
    counts a 4-byte action read; the on-device random policy reads no action.

    Z here is the observable zone block (zone ids are drawn in [0,4) whatever num_zones
    is, loadbalancer_k8s_env.py:354), i.e. the survey's Z=4 default.
    """
    E = cfg.num_endpoints
    Z = min(cfg.num_zones, 4) if cfg.num_zones >= 4 else cfg.num_zones
    b = 53 * E + 6 * Z + (240 if cfg.rejection_allowed else 208)
    return b if reads_actions else b - 4


def parse(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=100)  # one ring cycle: every timed launch is a full one
    ap.add_argument("--envs", type=int, default=1 << 20, help="envs in total (per GPU with --weak)")
    ap.add_argument("--weak", action="store_true", help="--envs per GPU (weak scaling)")
    ap.add_argument("--config", default="default", choices=sorted(CONFIGS))
    ap.add_argument("--ring", type=int, default=100,
                    help="rollout ring depth (obs slots; PPO's T = 100 storage, SURVEY 8d); lb_rollout launches fill it")
    ap.add_argument("--no-graph", action="store_true", help="launch every step eagerly")
    ap.add_argument("--launch", default="rollout", choices=("rollout", "step"),
                    help="rollout: K = ring steps per lb_rollout launch; step: one lb_step per step")
    ap.add_argument("--no-step-line", action="store_true", help="rollout mode: skip the lb_step measurement")
    ap.add_argument("--lockstep", action="store_true", help="do not stagger episodes (all envs reset together)")
    ap.add_argument("--geometry", default="auto", choices=("auto", "tpe", "slice"), help="E <= 8 kernel shape")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--plan-only", action="store_true", help="launcher + sharding + stats reduction, no GPU")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    return ap.parse_args(argv)


def cpu_baseline(cfg_kwargs, seconds):
    """The C oracle (Philox mode, OpenMP over envs) on a bounded sample of the same workload,
    plus the reference's process pattern (SubprocVecEnv: one worker process per core, one
    Pipe round trip per vector step) around the same oracle, one env per worker."""
    import numpy as np

    from oracle import oracle
    B = 1 << 16
    orc = oracle.OracleBatch(cfg_kwargs, B, trace=False, seed=0)
    orc.init()
    orc.reset()
    for _ in range(3):
        orc.step(orc.policy_random())
    steps = 0
    t0 = time.perf_counter()
    while True:
        a = orc.policy_random()
        orc.step(a)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    _ = np.zeros(1)
    out = dict(value=B * steps / el, unit="env-steps/s", cores=oracle.num_threads(), kind="port",
               sample=f"C oracle (oracle/lbk8s_oracle.c, OpenMP), {B} envs x {steps} vector steps "
                      f"({el:.1f} s), same scenario, Philox seed 0, random policy")
    try:
        out["subproc_vecenv"] = oracle.subproc_vecenv_rate(cfg_kwargs, workers=min(16, os.cpu_count() or 1),
                                                           seconds=min(5.0, seconds))
    except Exception as e:  # noqa: BLE001  (context only; never fails the bench)
        out["subproc_vecenv"] = {"error": repr(e)}
    out["reference_itself"] = {"value": REFERENCE_SUBPROC_8CORE, "cores": 8,
                               "sample": "the reference env under an 8-worker pipe VecEnv, survey container "
                                         "(BASELINE.md; the reference does not travel to the GPU box)"}
    return out


def plan_only(args, rank, world):
    """CPU path of the launcher: shard table and one episode-statistics all_reduce (gloo)."""
    import torch
    import torch.distributed as dist

    from lbk8s.dist import reduce_episode_stats, shard
    if world > 1:
        dist.init_process_group("gloo")
    off, n = shard(args.envs * (world if args.weak else 1), rank, world)
    # a fake ep_stats block: every env of this rank finished one episode of return = its global id
    st = torch.zeros((n, 16), dtype=torch.float64)
    st[:, 0] = torch.arange(off, off + n, dtype=torch.float64)
    st[:, 1] = 100.0
    red = reduce_episode_stats(st, torch.ones(n, dtype=torch.bool))
    shards = [None] * world
    if world > 1:
        dist.all_gather_object(shards, (rank, off, n))
    else:
        shards = [(rank, off, n)]
    if rank == 0:
        print(json.dumps({"plan": True, "world": world, "shards": shards,
                          "reduced": [float(x) for x in red]}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world_env == 1:
        # launch the ranks ourselves (before any GPU call), wait, and report their status
        from lbk8s.dist import launch
        raise SystemExit(launch(args.gpus, os.path.abspath(__file__), argv))
    if world_env != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = world_env
    if args.plan_only:
        return plan_only(args, rank, world)

    import torch
    import torch.distributed as dist

    from lbk8s import LBVecEnv
    from lbk8s.dist import shard
    from lbk8s.info import ST_EPISODE
    # one GPU per rank over RCCL; LBK8S_DIST_BACKEND=gloo (a test mode) lets ranks share GPUs
    backend = os.environ.get("LBK8S_DIST_BACKEND", "nccl")
    ngpu = torch.cuda.device_count()
    if backend == "nccl" and ngpu < world:
        raise SystemExit(f"bench.py: {world} ranks but {ngpu} visible GPUs")
    dev = torch.device("cuda", local % max(ngpu, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    total = args.envs * (world if args.weak else 1)
    off, B = shard(total, rank, world)
    cfg_kwargs = CONFIGS[args.config]
    env = LBVecEnv(B, device=dev, seed=0, env_id_offset=off, as_tensors=True, geometry=args.geometry, **cfg_kwargs)
    R = env.cfg.obs_rows
    L = env.cfg.episode_length
    T = max(1, args.ring)
    obs_ring = torch.empty((T, B, R, 8), dtype=torch.float32, device=dev)
    rew_ring = torch.empty((T, B), dtype=torch.float32, device=dev)
    done_ring = torch.empty((T, B), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def one_step(i):  # actions=None: the env's random policy, drawn inside the step kernel
        env.step_device(None, obs_out=obs_ring[i % T], reward_out=rew_ring[i % T], done_out=done_ring[i % T])

    launched = []  # vector steps per launch issued by run() (graph replays count their launches)

    def one_launch(mode, i, end, record=True):  # -> vector steps launched from step i
        if mode == "step":
            one_step(i)
            n = 1
        else:
            n = min(T - i % T, end - i)  # K = the ring's remaining slots: T steps per launch
            env.rollout("random", n, obs_out=obs_ring[i % T], reward_out=rew_ring[i % T], done_out=done_ring[i % T])
        if record:
            launched.append(n)
        return n

    # setup: stagger the episodes so 1/L of the envs end (and auto-reset) at every step
    env.reset()
    gid = torch.arange(off, off + B, device=dev)
    for r in range(1, 1 if args.lockstep else L):
        one_step(0)
        env.reset_masked((gid % L) == r)

    def measure(mode):
        # one graph of T steps (ring slots 0..T-1): no host launch cost between the kernels
        graph = None
        if not args.no_graph:
            side = torch.cuda.Stream(dev)
            side.wait_stream(stream)
            with torch.cuda.stream(side):
                one_step(0)
            stream.wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            graph_launches = []
            with torch.cuda.graph(graph):
                i = 0
                while i < T:
                    n = one_launch(mode, i, T, record=False)
                    graph_launches.append(n)
                    i += n

        def run(first, count):
            i, end = first, first + count
            while i < end:
                if graph is not None and i % T == 0 and end - i >= T:
                    graph.replay()
                    launched.extend(graph_launches)
                    i += T
                else:
                    i += one_launch(mode, i, end)

        K = args.steps
        # the timed window's launches not covered by whole ring cycles (a window that starts
        # or ends mid-ring, e.g. the driver's --warmup 5 --steps 20: one 20-step launch) are
        # captured as a graph of their own beforehand, so every timed launch is issued by a
        # graph replay instead of a host-side launch call (the same kernels and arguments).
        # Captured BEFORE the warm-up runs, so the warm-up's launches run right before the
        # timed window (capturing after them left the GPU idle for the capture: the timed
        # 20-step launch then ran ~8% slower than the same launch issued back to back)
        seg = None
        if not args.no_graph and (args.warmup % T != 0 or K % T != 0):
            seg = torch.cuda.CUDAGraph()
            seg_launches = []
            with torch.cuda.graph(seg):
                i, end = args.warmup, args.warmup + K
                while i < end:
                    n = one_launch(mode, i, end, record=False)
                    seg_launches.append(n)
                    i += n
        run(0, args.warmup)
        del launched[:]
        # resets in the window: the done flags of the K timed steps when they all still sit in
        # the ring afterwards (K <= T); otherwise the episode counters before and after.  (An
        # env.stats() pass right before the window -- 134 MB written at 2^20 envs -- evicted
        # the env state from the 256 MB Infinity Cache and slowed the timed 20-step launch 7%.)
        ring_count = K <= T
        ep0 = None if ring_count else env.stats()[:, ST_EPISODE].sum().item()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # timed: exactly K steps, barrier + synchronize on both sides; HIP events on the
        # kernels' stream bracket the same launches (their average = the kernel's duration)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        if seg is not None:
            seg.replay()
            launched.extend(seg_launches)
        else:
            run(args.warmup, K)
        ev1.record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        own_el = el
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        kernel_ms = ev0.elapsed_time(ev1) / K
        if ring_count:
            # (a done flag is a reset only under the VecEnv auto-reset; without it the window's
            # resets would be the ST_EPISODE count below)
            assert env.auto_reset, "ring reset count needs auto_reset"
            slots = [(args.warmup + j) % T for j in range(K)]
            resets = int(done_ring[slots].to(torch.int64).sum().item())
        else:
            resets = int(env.stats()[:, ST_EPISODE].sum().item() - ep0)
        assert env.status() == 0, "kernel flagged bad actions / unreset envs"
        assert kernel_ms <= own_el / K * 1e3 * 1.001, "event window longer than the wall-clock window"
        if world > 1:
            v = torch.tensor([float(resets)], dtype=torch.float64, device=dev)
            dist.all_reduce(v)
            resets = int(v[0].item())
        del graph, seg
        return dict(el=el, kernel_ms=kernel_ms, resets=resets, graphs=not args.no_graph, launches=list(launched))

    K = args.steps
    res = measure(args.launch)
    step_res = measure("step") if args.launch == "rollout" and not args.no_step_line else None
    el, kernel_ms, resets = res["el"], res["kernel_ms"], res["resets"]
    launches = res["launches"]
    assert sum(launches) == K, (launches, K)
    value = total * K / el
    b_step = algorithmic_bytes(env.cfg, reads_actions=False)
    out_b = 32 * R + 5  # obs rows + reward + done, written every step
    # byte model: lb_step moves b_step per env-step; an lb_rollout launch of k steps
    # writes out_b per env-step and reads + writes the state once: b_step - out_b per env per
    # launch.  Priced on the launches the timed window actually issued.
    n_launch = len(launches)
    k_avg = K / n_launch
    if args.launch == "step":
        b_alg, model = b_step, f"lb_step: {b_step} B per env-step (SURVEY 8d: 53E + 6Z + 236)"
    else:
        b_alg = out_b + (b_step - out_b) * n_launch / K
        model = f"lb_rollout: {out_b} + {b_step - out_b}/k B per env-step, k = {launches[0] if len(set(launches)) == 1 else launches} steps per launch"
    achieved = b_alg * B / (kernel_ms * 1e-3) / 1e9
    traffic = None
    # PMC passes per launch shape: pmc_traffic.json (lb_step), pmc_traffic_rollout_k{K}.json
    # (lb_rollout launches of K steps); only a pass of the same shape (config, envs, steps per
    # launch) prices this line, otherwise traffic is null
    if args.launch == "step":
        pmc_paths = [args.pmc_json]
    else:
        pmc_paths = [args.pmc_json.replace(".json", f"_rollout_k{launches[0]}.json"),
                     args.pmc_json.replace(".json", "_rollout.json")]
    pmc_file = None
    for pmc_path in pmc_paths:
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
        except (OSError, ValueError):
            continue
        if (pmc.get("config") == args.config and pmc.get("envs") == B and len(set(launches)) == 1
                and pmc.get("steps_per_launch", 1) == launches[0]):
            traffic = pmc.get("hbm_bytes_per_launch")
            pmc_file = os.path.relpath(pmc_path, REPO)
            break
    tpe = env.cfg.num_endpoints <= 8 and (args.geometry == "tpe" or (args.geometry == "auto" and B >= 32768))
    if args.launch == "step":
        kname = "k_step_tpe (lb_step, auto-reset inside)" if tpe else "k_step_slice (lb_step)"
    else:
        # the kernel lb_rollout picks for this launch shape (lb_rollout_kernel, host only)
        kname = f"{env.rollout_kernel(launches[0])} (lb_rollout, random policy, auto-reset inside)"
    line = {
        "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": K,
        "warmup": args.warmup, "ms_per_step": el / K * 1e3, "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (Philox seed 0 scenarios; the env's uniform random policy drawn on the device)",
        "config": {"workload": f"config 3: {total} {args.config}-scenario envs in total "
                               f"(E={env.cfg.num_endpoints}, N={env.cfg.num_nodes}, Z={env.cfg.num_zones}, "
                               f"{env.cfg.reward_function}), {B} per GPU, obs ring T={T}, "
                               + ("lockstep" if args.lockstep else "staggered") + " episodes, "
                               + (f"timed as {n_launch} lb_rollout launch(es) of {launches} vector steps"
                                  if args.launch == "rollout" else "one lb_step launch per vector step"),
                   "envs_per_gpu": B, "total_envs": total, "scenario": args.config, "episode_length": L,
                   "resets_in_window": resets, "graphs": res["graphs"], "geometry": args.geometry,
                   "launch": args.launch, "parallelism": f"env-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": pmc_file, "kernel": kname,
                     "kernel_ms": kernel_ms, "bytes_per_env_step": b_alg, "byte_model": model,
                     "envs_per_launch": B, "launches_timed": n_launch, "steps_per_launch": k_avg,
                     # one launch = steps_per_launch vector steps: the rocprof average duration
                     # of the kernel is launch_ms; traffic is HBM bytes per launch (PMC, same k)
                     "launch_ms": kernel_ms * k_avg,
                     "traffic_bytes_per_env_step": (traffic / B / k_avg if traffic is not None else None),
                     # the same time against SURVEY 8(d)'s per-env-step bytes of the one-launch-
                     # per-step design (the rollout moves fewer: frac > 1 there means it beats
                     # that design's bandwidth bound), and against the PMC-measured bytes
                     "frac_at_survey_bytes": b_step * B / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "frac_measured_traffic": (traffic / k_avg / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                               if traffic is not None else None)},
    }
    if step_res is not None:
        ks = step_res["kernel_ms"]
        line["lb_step"] = {"value": total * K / step_res["el"], "ms_per_step": step_res["el"] / K * 1e3,
                           "kernel_ms": ks, "bytes_per_env_step": b_step,
                           "frac": b_step * B / (ks * 1e-3) / 1e9 / HBM_PEAK_GBS,
                           "kernel": "k_step_tpe (lb_step, auto-reset inside)" if tpe else "k_step_slice (lb_step)",
                           "resets_in_window": step_res["resets"]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(cfg_kwargs, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
