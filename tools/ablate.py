#!/usr/bin/env python3
"""A/B the perf-experiment builds of liblbk8s (tools/_build/liblbk8s_<variant>.so) in ONE
process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).  Obs ring 16.
Prints median/min ms per lb_step per variant.

    python tools/ablate.py [variants,comma,separated] [scenario (bench.CONFIGS)] [envs]"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]

import torch  # noqa: E402

from lbk8s import LBConfig, _native  # noqa: E402


def load(path):
    L = C.CDLL(path)
    vp, i64 = C.c_void_p, C.c_int64
    cfgp = C.POINTER(_native.LBConfigC)
    L.lb_state_bytes.argtypes = [cfgp, i64, C.POINTER(C.c_uint64)]
    L.lb_init.argtypes = [vp, cfgp, i64, vp, vp]
    L.lb_reset.argtypes = [vp, cfgp, i64, vp, vp, vp, vp]
    L.lb_step.argtypes = [vp, cfgp, i64, vp, vp, vp, vp, vp, vp, vp, vp]
    return L


def main():
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["base", "PLAIN_OBS", "NO_LUT", "NO_OBS", "NO_RNG", "ED_FULL", "NT_STATE", "NT_LOAD"]
    scenario = sys.argv[2] if len(sys.argv) > 2 else "default"
    from bench import CONFIGS
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
    dev = torch.device("cuda", 0)
    cfg = LBConfig(**CONFIGS[scenario])
    c = cfg.to_c(seed=0)
    R, T = cfg.obs_rows, 16
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    libs = {n: load(os.path.join(REPO, "tools", "_build", f"liblbk8s_{n}.so")) for n in names}
    n = C.c_uint64()
    libs[names[0]].lb_state_bytes(C.byref(c), B, C.byref(n))
    ring = torch.empty((T, B, R, 8), dtype=torch.float32, device=dev)
    rew = torch.empty((T, B), dtype=torch.float32, device=dev)
    dn = torch.empty((T, B), dtype=torch.uint8, device=dev)
    term = torch.empty((B, R, 8), dtype=torch.float32, device=dev)
    st = torch.empty((B, 16), dtype=torch.float64, device=dev)
    acts = torch.randint(0, cfg.num_actions, (32, B), dtype=torch.int32, device=dev)
    states = {}
    for name, L in libs.items():
        s = torch.zeros(n.value, dtype=torch.uint8, device=dev)
        assert L.lb_init(s.data_ptr(), C.byref(c), B, None, stream) == 0
        assert L.lb_reset(s.data_ptr(), C.byref(c), B, None, ring[0].data_ptr(), None, stream) == 0
        states[name] = s
    res = {k: [] for k in names}
    i = 0
    for rnd in range(6):
        for name, L in libs.items():
            s = states[name]
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for w in range(5):
                L.lb_step(s.data_ptr(), C.byref(c), B, acts[i % 32].data_ptr(), ring[i % T].data_ptr(),
                          rew[i % T].data_ptr(), dn[i % T].data_ptr(), term.data_ptr(), st.data_ptr(), None, stream)
                i += 1
            ev0.record()
            for w in range(40):
                L.lb_step(s.data_ptr(), C.byref(c), B, acts[i % 32].data_ptr(), ring[i % T].data_ptr(),
                          rew[i % T].data_ptr(), dn[i % T].data_ptr(), term.data_ptr(), st.data_ptr(), None, stream)
                i += 1
            ev1.record()
            torch.cuda.synchronize()
            res[name].append(ev0.elapsed_time(ev1) / 40)
    for name in names:
        v = sorted(res[name])
        print(json.dumps(dict(variant=name, scenario=scenario, envs=B, median_ms=round(v[len(v) // 2], 5), min_ms=round(v[0], 5),
                              env_steps_per_s=B / v[len(v) // 2] * 1e3)))


if __name__ == "__main__":
    main()
