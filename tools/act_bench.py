#!/usr/bin/env python3
"""The DQN vector step's action launch (lb_dqn_act: explore decision + fused Q forward and
masked argmax) at config 5's shape, replayed from a HIP graph of --n launches.

    python tools/act_bench.py [--envs 4096] [--n 50] [--reps 5] [--lib exp/x.so]

One JSON line per (lib, mode): microseconds per launch for the greedy path (epsilon 0),
the explore path (epsilon 1) and lb_ds_q_argmax (no decision), and the actions' checksum
(the A/B builds must agree).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--n", type=int, default=50)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--vector-step", action="store_true",
                    help="time the whole DQN vector step: lb_dqn_step vs act + step + replay add")
    args = ap.parse_args()
    from lbk8s import _native
    if args.lib:
        _native.LIB_PATH = os.path.abspath(args.lib)
    import ctypes as C

    import torch

    from lbk8s import LBVecEnv, fused
    from lbk8s.deepsets import DQNDeepSetAgent
    torch.manual_seed(0)
    env = LBVecEnv(args.envs, device="cuda", seed=3)
    env.reset()
    obs = env.obs.clone()
    B, R = obs.shape[0], obs.shape[1]
    agent = DQNDeepSetAgent(env).cuda()
    frag = fused.frag_buffer(obs.device)
    fused.pack_q_into(agent, frag)
    masks = torch.ones((B, R), dtype=torch.bool, device="cuda")
    act = torch.zeros(B, dtype=torch.int32, device="cuda")
    vpp = torch.zeros(2, dtype=torch.int64, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    L = _native.lib()
    exs = {eps: _native.LBDQNExploreC(eps, 0.0, eps, 12345, vpp.data_ptr(), vpp.data_ptr() + 8, flag.data_ptr())
           for eps in (0.0, 1.0)}

    from lbk8s.dqn import DeviceReplayBuffer
    rb = DeviceReplayBuffer(16 * B, B, (R, 8), obs.device, None)
    nxt, rew = torch.empty_like(obs), torch.empty(B, device="cuda")
    dn = torch.empty(B, dtype=torch.uint8, device="cuda")
    es, ec = torch.zeros(B, dtype=torch.float64, device="cuda"), torch.zeros(B, dtype=torch.float64, device="cuda")
    m8 = masks.to(torch.uint8)

    def launch(mode):
        st = torch.cuda.current_stream().cuda_stream
        ex = exs[1.0 if mode.endswith("explore") else 0.0]
        pp = rb.pos_pp.data_ptr()
        if mode.startswith("step3"):  # the vector step as three launches: act, env step, replay write
            env.dqn_act(frag, obs, m8, ex, act)
            env.step_device(act, obs_out=nxt, reward_out=rew, done_out=dn)
            rb.add_fused(obs, nxt, act, rew, dn, env.ep_stats, es, ec, 0)
            return
        if mode.startswith("dqn_step"):  # lb_dqn_step (one launch at config 5's shape)
            env.dqn_step(frag, obs, m8, ex, act, nxt, rew, dn, rb, pp, pp + 8, es, ec)
            return
        if mode == "q_argmax":
            _native.check(L.lb_ds_q_argmax(frag.data_ptr(), obs.data_ptr(), B, R, masks.data_ptr(), None,
                                           act.data_ptr(), st))
        else:
            env.dqn_act(frag, obs, masks, exs[0.0 if mode == "greedy" else 1.0], act)

    lib = os.path.basename(_native.LIB_PATH)
    modes = ("greedy", "explore", "q_argmax") if not args.vector_step else \
        ("step3_greedy", "dqn_step_greedy", "step3_explore", "dqn_step_explore")
    for mode in modes:
        launch(mode)
        torch.cuda.synchronize()
        side = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                for _ in range(args.n):
                    launch(mode)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        us = []
        for _ in range(args.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            torch.cuda.synchronize()
            us.append(1e3 * s.elapsed_time(e) / args.n)
        print(json.dumps({"lib": lib, "mode": mode, "envs": B, "R": R, "us_per_launch": round(min(us), 2),
                          "us_all": [round(u, 2) for u in us], "actions_sum": int(act.long().sum())}), flush=True)


if __name__ == "__main__":
    main()
