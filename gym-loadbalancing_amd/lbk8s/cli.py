"""run.py equivalent: the reference's CLI on the MI355X framework.

    python -m lbk8s.cli --alg ppo_deepsets --num_endpoints 64 --num_envs 4096 --total_steps 409600

Same flags and defaults as /root/reference/run.py:23-45, the same env construction
(get_env, :95-127: arrival rate 100, call duration 1, episode length 100, latency weight
1, cpu 0, gini 0; rejection only with --rejection), the same trainer arguments
(get_model, :54-72) and the same model name (:189-191).  By design:
  * the reference's SubprocVecEnv of 8 workers becomes one LBVecEnv of --num_envs envs
    (default 8) on the GPU, trained by the GPU-resident lbk8s.ppo / lbk8s.dqn;
  * only the deep-sets algorithms exist here: "ppo", "a2c", "recurrent_ppo" and
    "mask_ppo" (:56-63) are stable-baselines3 models, which this framework does not
    include (LBVecEnv can serve them as a VecEnv);
  * --testing runs the greedy evaluation of lbk8s.evaluate on the saved / given
    checkpoint (the reference's test_model, :130-161, plots one episode's reward);
  * loading returns the agent (the reference's get_load_model returns load()'s None);
  * the training envs write VecMonitor's file, vec_loadbalancer_k8s_gym_results.monitor.csv
    (run.py:122; one file per rank, suffixed, with --nproc > 1);
  * --nproc N trains on N GPUs of the node: N ranks (one process per GPU, launched here
    through torch.distributed.run), each with --num_envs envs of its own global env-id
    range, gradients and episode statistics all-reduced over RCCL; rank 0 saves.
"""
import argparse
import json
import logging
import os
import sys

SB3_ALGS = ("ppo", "recurrent_ppo", "a2c", "mask_ppo")


def build_parser():
    p = argparse.ArgumentParser(description="Run RL Agent!")
    p.add_argument("--alg", default="dqn_deepsets",
                   help='The algorithm: ["mask_ppo", "recurrent_ppo", "ppo", "mask_ppo", "ppo_deepsets", "dqn_deepsets"]')
    p.add_argument("--env_name", default="loadbalancer", help='Env: ["loadbalancer"]')
    p.add_argument("--num_endpoints", default=6, help="num_endpoints: 4, 8, etc")
    p.add_argument("--rejection", default=False, action="store_true", help="Testing mode")
    p.add_argument("--num_zones", default=4, help="num_zones: 4, 8, etc")
    p.add_argument("--num_nodes", default=24, help="num_nodes: 4, 8, etc")
    p.add_argument("--reward", default="multi", help='reward: ["naive", "latency", "fairness", "multi"]')
    p.add_argument("--training", default=True, action="store_true", help="Training mode")
    p.add_argument("--testing", default=False, action="store_true", help="Testing mode")
    p.add_argument("--loading", default=False, action="store_true", help="Loading mode")
    p.add_argument("--load_path",
                   default="results/a2c/multi/"
                           "ppo_env_loadbalancer_num_endpoints_6_num_zones_4_reward_multi_totalSteps_200000_run_1/"
                           "ppo_env_loadbalancer_num_endpoints_6_num_zones_4_reward_multi_totalSteps_200000",
                   help="Loading path, ex: logs/model/test.zip")
    p.add_argument("--test_path",
                   default="results/loadbalancer/multi/"
                           "a2c_env_loadbalancer_num_endpoints_6_num_zones_4_reward_multi_totalSteps_200000_run_1/"
                           "a2c_env_loadbalancer_num_endpoints_6_num_zones_4_reward_multi_totalSteps_200000",
                   help="Testing path, ex: logs/model/test.zip")
    p.add_argument("--steps", default=200000, help="Save model after X steps")
    p.add_argument("--total_steps", default=200000, help="The total number of steps.")
    # framework additions
    p.add_argument("--num_envs", default=8, type=int, help="parallel envs on the GPU (reference: 8 workers)")
    p.add_argument("--no_training", action="store_true", help="skip training (--training is always on)")
    p.add_argument("--test_episodes", default=1, type=int, help="episodes played side by side by --testing")
    p.add_argument("--test_sequential", action="store_true",
                   help="--testing plays the episodes one after another on one env, as run_test_deepset.py")
    p.add_argument("--device", default="cuda")
    p.add_argument("--seed", default=0, type=int, help="Philox seed of the envs")
    p.add_argument("--nproc", default=1, type=int, help="GPUs (ranks) to train on, one process each")
    p.add_argument("--monitor_file", default="vec_loadbalancer_k8s_gym_results",
                   help="VecMonitor file of the training envs (run.py:122); '' disables it")
    return p


def env_kwargs(rejection, num_endpoints, num_zones, num_nodes, reward_function):
    """get_env's LoadBalancerK8sEnv arguments (run.py:97-107)."""
    return dict(num_nodes=num_nodes, num_zones=num_zones, num_endpoints=num_endpoints,
                rejection_allowed=rejection, arrival_rate_r=100, call_duration_r=1, episode_length=100,
                reward_function=reward_function, latency_weight=1.0, cpu_weight=0.0, gini_weight=0.0)


def get_env(env_name, rejection, num_endpoints, num_zones, num_nodes, reward_function, num_envs=8,
            device="cuda", seed=0, env_id_offset=0, monitor_file=None):
    if env_name != "loadbalancer":
        raise SystemExit("Invalid environment!")
    from .info import INFO_KEYS
    from .vec_env import LBVecEnv
    return LBVecEnv(num_envs, device=device, seed=seed, env_id_offset=env_id_offset, as_tensors=True, monitor=True,
                    info_keywords=INFO_KEYS, monitor_file=monitor_file or None,
                    **env_kwargs(rejection, num_endpoints, num_zones, num_nodes, reward_function))


def get_model(alg, env, rank=0):
    """get_model (run.py:54-72) for the deep-sets algorithms.  With several ranks each rank's
    learner seed is offset by its rank, so rollout uniforms, minibatch permutations, replay
    samples and exploration coins differ across GPUs (the parameters are broadcast from rank
    0, so the replicas still start identical)."""
    if alg == "ppo_deepsets":
        from .ppo import PPO_DeepSets
        return PPO_DeepSets(env, num_steps=100, n_minibatches=8, ent_coef=0.001, seed=2 + rank)
    if alg == "dqn_deepsets":
        from .dqn import DQN_DeepSets
        return DQN_DeepSets(env, num_steps=100, n_minibatches=8, seed=1 + rank)
    if alg in SB3_ALGS:
        raise SystemExit(f"{alg!r} is a stable-baselines3 model; this framework provides the deep-sets "
                         "algorithms (ppo_deepsets, dqn_deepsets) and LBVecEnv as a VecEnv")
    raise SystemExit("Invalid algorithm!")


def model_name(alg, env_name, num_endpoints, num_zones, reward, total_steps):
    """run.py:189-191."""
    return (alg + "_env_" + env_name + "_num_endpoints_" + str(num_endpoints) + "_num_zones_" + str(num_zones)
            + "_reward_" + reward + "_totalSteps_" + str(total_steps))


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = build_parser().parse_args(argv)
    if args.nproc > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        # spawn the ranks before anything touches the GPU, then wait for them
        from .dist import launch
        child = [a for i, a in enumerate(argv)  # the ranks get the torchrun environment instead
                 if not a.startswith("--nproc") and not (i > 0 and argv[i - 1] == "--nproc")]
        raise SystemExit(launch(args.nproc, "lbk8s.cli", child, module=True))
    logging.info(args)
    alg, reward = args.alg, args.reward
    num_nodes, num_zones, num_endpoints = int(args.num_nodes), int(args.num_zones), int(args.num_endpoints)
    total_steps = int(args.total_steps)
    name = model_name(alg, args.env_name, num_endpoints, num_zones, reward, total_steps)
    result = {"name": name}
    if args.training and not args.no_training:
        from .dist import init_from_env
        rank, world, dev = init_from_env("cuda" if str(args.device).startswith("cuda") else "cpu")
        mon = args.monitor_file + (f"_rank{rank}" if world > 1 and args.monitor_file else "")
        env = get_env(args.env_name, args.rejection, num_endpoints, num_zones, num_nodes, reward,
                      num_envs=args.num_envs, device=dev if world > 1 else args.device, seed=args.seed,
                      env_id_offset=rank * args.num_envs, monitor_file=mon)
        model = get_model(alg, env, rank)
        if args.loading:  # resume training
            model.load(args.load_path)
        model.learn(total_timesteps=total_steps)
        env.close()
        result.update(world_size=world, episode_returns=[float(r) for r in model.episode_returns[-3:]])
        if rank == 0:
            model.save(name)
            result["saved"] = name
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
            if rank != 0:
                return result
    if args.testing:
        from .evaluate import load_agent, run_sequential, run_test
        agent = load_agent(args.test_path, "ppo" if alg == "ppo_deepsets" else "dqn", device=args.device)
        kw = env_kwargs(args.rejection, num_endpoints, num_zones, num_nodes, reward)
        if args.test_sequential:
            from .vec_env import LBVecEnv
            env = LBVecEnv(1, device=args.device, seed=args.seed, as_tensors=True, **kw)
            res = run_sequential(agent, args.test_episodes, env)
        else:
            res = run_test(agent, n_episodes=args.test_episodes, seed=args.seed, device=args.device, **kw)
        result["test_returns"] = [float(r) for r in res["r"]]
    print(json.dumps(result))
    return result


if __name__ == "__main__":
    main()
