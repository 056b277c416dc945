#!/usr/bin/env python3
"""Learner benchmarks: SURVEY §8(d) configs 4 (PPO) and 5 (DQN), env-steps/s including updates.

    python tools/rl_bench.py --algo ppo [--envs 4096] [--updates 2] [--warmup-updates 1]
    python tools/rl_bench.py --algo dqn [--envs 4096] [--steps 2000] [--warmup 300]
    torchrun --nproc-per-node N tools/rl_bench.py --algo ppo ...    (RCCL gradient all-reduce)

Config 4: E=64, N=24, Z=4, rejection, multi (lw=1, cw=0, gw=0), B envs per GPU, PPO with
T=100, 8 minibatches, 4 epochs, ent_coef 0.001 (run.py), gamma 0.95, lambda 0.97,
Adam(2.5e-4, eps 1e-5), clip_grad_norm 0.5.  One timed update = rollout of T vector steps
(fused deep-sets forward + sampling + fused env step) + GAE + 32 minibatch steps.
Config 5: default scenario, B envs per GPU, DQN defaults (buffer 10,000 // B slots per env,
batch 128, train every 10 vector steps, target copy every 500, gamma 0.99), except
learning_starts: the warm-up phase fills the buffer and the timed phase trains at the
default frequency throughout.

One JSON line (rank 0): whole-job env-steps/s (= all ranks' env steps / max-over-ranks
time), the rollout / update split, and the run's last losses.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]

from bench import CONFIGS  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", choices=("ppo", "dqn"), default="ppo")
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS))
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--updates", type=int, default=2)
    ap.add_argument("--warmup-updates", type=int, default=1)
    ap.add_argument("--num-steps", type=int, default=100)
    ap.add_argument("--steps", type=int, default=2000, help="DQN timed vector steps")
    ap.add_argument("--warmup", type=int, default=300, help="DQN warm-up vector steps")
    ap.add_argument("--lib", default=None, help="another build of liblbk8s.so (an A/B across builds)")
    ap.add_argument("--torch-set-sums", action="store_true",
                    help="A/B reference: the training step's sums over the sets as round-5's chunked torch GEMMs "
                         "(fused_train._over_sets) instead of lb_ds_over_sets")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from lbk8s import LBVecEnv, _native, fused_train
    if args.lib:
        _native.LIB_PATH = os.path.abspath(args.lib)
    if args.torch_set_sums:
        def torch_sums(jobs, S, dev):
            out = []
            for a, b, scale in jobs:
                if a is None:
                    out.append((scale * b.sum(0, keepdim=True)) if scale != 1.0 else b.sum(0, keepdim=True))
                else:
                    out.append(fused_train._over_sets(a, b, scale))
            return out
        fused_train.sums_over_sets = torch_sums
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    B = args.envs
    name = args.config or ("e64_multi" if args.algo == "ppo" else "default")
    env = LBVecEnv(B, device=dev, seed=0, env_id_offset=rank * B, as_tensors=True, **CONFIGS[name])

    def barrier_sync():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    out = dict(algo=args.algo, config=name, envs_per_gpu=B, n_gpus=world)
    if args.algo == "ppo":
        from lbk8s.ppo import PPO_DeepSets
        ppo = PPO_DeepSets(env, num_steps=args.num_steps, n_minibatches=8, update_epochs=4, ent_coef=0.001,
                           gamma=0.95, gae_lambda=0.97, seed=1, device=dev)
        next_obs = env.reset()
        next_done = torch.zeros(B, device=dev)
        for _ in range(args.warmup_updates):
            next_obs, next_done = ppo.rollout(next_obs, next_done)
            ppo.update(next_obs, next_done)
        t_roll = t_upd = 0.0
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(args.updates):
            a = time.perf_counter()
            next_obs, next_done = ppo.rollout(next_obs, next_done)
            torch.cuda.synchronize(dev)
            b = time.perf_counter()
            stats = ppo.update(next_obs, next_done)
            torch.cuda.synchronize(dev)
            t_roll += b - a
            t_upd += time.perf_counter() - b
        barrier_sync()
        wall = max_over_ranks(time.perf_counter() - t0)
        env_steps = args.updates * args.num_steps * B * world
        out.update(metric="env-steps/s including PPO updates (config 4)", value=env_steps / wall,
                   unit="env-steps/s", updates=args.updates, num_steps=args.num_steps, minibatches=8, epochs=4,
                   ms_per_update=wall / args.updates * 1e3, rollout_ms=t_roll / args.updates * 1e3,
                   update_ms=t_upd / args.updates * 1e3,
                   rollout_env_steps_per_s=args.num_steps * B * world * args.updates / max_over_ranks(t_roll),
                   last=dict((k, round(v, 6)) for k, v in stats.items()),
                   ep_return=ppo.episode_returns[-1] if ppo.episode_returns else None)
    else:
        from lbk8s.dqn import DQN_DeepSets
        dqn = DQN_DeepSets(env, seed=1, learning_starts=min(100, args.warmup // 2), device=dev,
                           train_graph=os.environ.get("LBK8S_DQN_TRAIN_GRAPH", "1") == "1",  # (A/B switches)
                           period_graph=os.environ.get("LBK8S_DQN_PERIOD_GRAPH", "1") == "1",
                           device_rng=os.environ.get("LBK8S_DQN_DEVICE_RNG", "1") == "1")
        dqn.learn(args.warmup)
        # (the timed learn()'s period graphs captured beforehand: a one-time cost, amortised to
        # nothing over run.py's 500,000 steps; LBK8S_BENCH_PREPARE=0 times it as rounds 3-4 did)
        if os.environ.get("LBK8S_BENCH_PREPARE", "1") == "1":
            dqn.prepare(args.steps)
        barrier_sync()
        t0 = time.perf_counter()
        dqn.learn(args.steps)
        barrier_sync()
        wall = max_over_ranks(time.perf_counter() - t0)
        env_steps = args.steps * B * world
        out.update(metric="env-steps/s including DQN training (config 5)", value=env_steps / wall,
                   unit="env-steps/s", vector_steps=args.steps, train_steps=dqn.train_steps,
                   ms_per_vector_step=wall / args.steps * 1e3,
                   buffer_slots_per_env=dqn.rb.size, train_graph=dqn.train_graph,
                   period_graph=dqn.period_graph, device_rng=dqn.device_rng,
                   graphs_captured_before_timing=os.environ.get("LBK8S_BENCH_PREPARE", "1") == "1",
                   ep_return=dqn.episode_returns[-1] if dqn.episode_returns else None)
    out.update(lib=os.path.basename(_native.LIB_PATH), set_sums="torch" if args.torch_set_sums else "lb_ds_over_sets")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
