#!/usr/bin/env python3
"""Micro-bench of the fused deep-sets training kernels (one PPO minibatch's sets).

    python tools/train_bench.py [--sets 51200] [--R 65,9] [--iters 20] [--lib exp/x.so]

Times lb_ds_train_forward (actor + critic), lb_ds_train_backward (both heads + the
partial-sum reduce) with HIP events on the launch stream, and reports useful TFLOP/s
(FLOPs of the torch formulation at the true R) and the fraction of the
157.3 TFLOP/s f32 MFMA peak.  --lib runs another build of liblbk8s.so (A/B).
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]
PEAK = 157.3


def fwd_flops(R):
    # actor: 8->64, 64->64, 64->1 on R rows + pooled rows; critic: two layers + layer-3 and rho
    eq = lambda i, o: 2 * i * o * (R + 1)  # noqa: E731
    return eq(8, 64) + eq(64, 64) + eq(64, 1) + eq(8, 64) + eq(64, 64) + eq(64, 64) + 2 * 64 * 64 + 2 * 64


def bwd_flops(R):
    # per head: data gradient 64x64 on R rows + dLambda2 (64x64 over R rows) + dLambda1 (64x8)
    per = 2 * 64 * 64 * R + 2 * 64 * 64 * R + 2 * 64 * 8 * R
    return 2 * per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=51200)
    ap.add_argument("--R", default="65,9")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default=None)
    args = ap.parse_args()
    from lbk8s import _native
    if args.lib:
        _native.LIB_PATH = os.path.abspath(args.lib)
    import torch

    from lbk8s import fused
    from lbk8s.deepsets import DeepSetAgent
    L = _native.lib()
    torch.manual_seed(0)
    agent = DeepSetAgent(8).cuda()
    st = torch.cuda.current_stream().cuda_stream
    for R in (int(r) for r in args.R.split(",")):
        B = args.sets
        x = torch.rand(B, R, 8, device="cuda") * 3
        frag = fused.packed(agent, agent.actor.net, agent.critic)
        w, keep = fused._weights_struct(agent.actor.net, agent.critic)
        bfrag = torch.empty(_native.LB_DS_BWD_FLOATS, device="cuda")
        _native.check(L.lb_ds_pack_backward(C.byref(w), bfrag.data_ptr(), st))
        logits = torch.empty(B, R, device="cuda")
        mean = torch.empty(B, 64, device="cuda")
        sa = torch.empty(2, B, R, 64, device="cuda")
        sc = torch.empty(2, B, R, 64, device="cuda")
        dl = torch.randn(B, R, device="cuda") * 1e-3
        dm = torch.randn(B, 64, device="cuda") * 1e-3
        wg = torch.empty(2, _native.LB_DS_WGRAD_FLOATS, device="cuda")
        work = torch.empty(_native.LB_DS_WORKSPACE_FLOATS, device="cuda")
        sv = torch.empty(B, _native.LB_DS_SETVEC_FLOATS, device="cuda")

        def f():
            _native.check(L.lb_ds_train_forward(frag.data_ptr(), x.data_ptr(), B, R, logits.data_ptr(),
                                                mean.data_ptr(), sa.data_ptr(), sc.data_ptr(), sv.data_ptr(), st))

        def b():
            _native.check(L.lb_ds_train_backward(bfrag.data_ptr(), x.data_ptr(), B, R, sa.data_ptr(), sc.data_ptr(),
                                                 dl.data_ptr(), dm.data_ptr(), wg.data_ptr(), work.data_ptr(),
                                                 sv.data_ptr(), st))

        def timed(fn):
            for _ in range(3):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(args.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            return s.elapsed_time(e) / args.iters

        f()
        fm, bm = timed(f), timed(b)
        ft, bt = fwd_flops(R) * B / fm / 1e9, bwd_flops(R) * B / bm / 1e9
        print(json.dumps(dict(sets=B, R=R, fwd_ms=round(fm, 4), fwd_tflops=round(ft, 1), fwd_frac=round(ft / PEAK, 3),
                              bwd_ms=round(bm, 4), bwd_tflops=round(bt, 1), bwd_frac=round(bt / PEAK, 3),
                              wgrad_checksum=float(wg.double().abs().sum()),
                              lib=os.path.basename(args.lib or _native.LIB_PATH))), flush=True)


if __name__ == "__main__":
    main()
