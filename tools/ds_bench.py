#!/usr/bin/env python3
"""Fused deep-sets forward (lb_ds_forward) vs the torch modules on the same GPU.

    python tools/ds_bench.py [--cases 8x9,4096x65,65536x9,1048576x9] [--iters 50]

One JSON line per case: fused and torch ms per forward (actor logits + critic value),
algorithmic TFLOP/s (the torch formulation's FLOPs: Lambda on every element, Gamma on
the pooled row, rho once) and the fraction of the f32 MFMA peak (157.3 TFLOP/s,
MI355X_MICROARCH.md).  Also checks the two agree (rtol 1e-4).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]

F32_MFMA_PEAK_TFLOPS = 157.3


def flops_per_env(R, C=8, H=64):
    eq = lambda i, o: 2 * i * o * (R + 1)  # noqa: E731  (Lambda on R rows + Gamma on the pooled row)
    actor = eq(C, H) + eq(H, H) + eq(H, 1)
    critic = eq(C, H) + eq(H, H) + eq(H, H) + 2 * H * H + 2 * H
    return actor + critic


def timed(fn, iters):
    import torch
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="8x9,4096x65,65536x9,1048576x9")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-torch", action="store_true")
    args = ap.parse_args()
    import torch

    from lbk8s import fused
    from lbk8s.deepsets import DeepSetAgent
    torch.manual_seed(0)
    agent = DeepSetAgent(8).cuda()
    for case in args.cases.split(","):
        B, R = (int(v) for v in case.split("x"))
        x = torch.rand(B, R, 8, device="cuda")
        fused_ms = timed(lambda: fused.deepsets_forward(agent, x, require=True), args.iters)
        out = dict(case=f"B={B} R={R}", fused_ms=round(fused_ms, 4), env_forwards_per_s=B / fused_ms * 1e3)
        fl = flops_per_env(R) * B
        out["algorithmic_tflops"] = fl / fused_ms / 1e9
        out["frac_f32_mfma_peak"] = out["algorithmic_tflops"] / F32_MFMA_PEAK_TFLOPS
        if not args.no_torch:
            with torch.no_grad():
                torch_ms = timed(lambda: (agent.actor(x), agent.critic(x)), args.iters)
                lt, vt = agent.actor(x), agent.critic(x)
            lf, vf = fused.deepsets_forward(agent, x, require=True)
            out.update(torch_ms=round(torch_ms, 4), speedup=torch_ms / fused_ms,
                       max_rel_err=float(max(((lf - lt).abs() / (lt.abs() + 1e-3)).max(),
                                             ((vf - vt).abs() / (vt.abs() + 1e-3)).max())))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
