#!/usr/bin/env python3
"""Where a k_rollout_lean step's time goes (diagnostic build with -DLB_TIMELINE:
exp/liblbk8s_timeline.so).  Each wave's lane 0 stamps s_memtime at 6 points of every step:
  0 step start | 1 after apply (+ ballot) | 2 after the auto-reset path | 3 stage 0 of the
  stores (the next step's gathers and record prefetch issued) | 4 every store issued |
  5 the gathers landed (the counted wait)
and s_memrealtime (100 MHz) at the launch start / end of the wave, to convert.  Prints the mean
cycles of each interval over waves and steps (steps 1..K-2), and the wave lifetime.

    python tools/timeline_lean.py --lib exp/liblbk8s_timeline.so --steps 20
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]
NP = 6
NH = 8  # header: loop start, loop end, entry, exit, records drawn, image built (realtime), HW_ID, XCC_ID


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="exp/liblbk8s_timeline.so")
    ap.add_argument("--envs", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lockstep", action="store_true")
    ap.add_argument("--save", default=None, help="write the raw per-wave stamps (npz) here")
    args = ap.parse_args()
    import numpy as np
    import torch

    from lbk8s import LBVecEnv, _native
    _native.LIB_PATH = os.path.abspath(args.lib)
    L = _native.lib()
    L.lbx_set_timeline.argtypes = [C.c_void_p]
    B, K = args.envs, args.steps
    env = LBVecEnv(B, seed=0, as_tensors=True)
    assert env.rollout_kernel(K).startswith("k_rollout_lean")
    R, EL = env.cfg.obs_rows, env.cfg.episode_length
    T = 100
    obs = torch.empty((T, B, R, 8), dtype=torch.float32, device="cuda")
    rew = torch.empty((T, B), dtype=torch.float32, device="cuda")
    done = torch.empty((T, B), dtype=torch.uint8, device="cuda")
    env.reset()
    gid = torch.arange(B, device="cuda")
    for r in range(1, 1 if args.lockstep else EL):
        env.step_device(None, obs_out=obs[0], reward_out=rew[0], done_out=done[0])
        env.reset_masked((gid % EL) == r)
    waves = B // 64
    tl = torch.zeros((waves, NH + K * NP), dtype=torch.int64, device="cuda")
    out = {}
    for i in range(4):
        if i == 3:
            assert L.lbx_set_timeline(tl.data_ptr()) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.rollout("random", K, obs_out=obs[i * K % (T - K + 1)], reward_out=rew[i * K % (T - K + 1)],
                    done_out=done[i * K % (T - K + 1)])
        e1.record()
        torch.cuda.synchronize()
        out[f"launch{i}_us"] = round(e0.elapsed_time(e1) * 1e3, 1)
    assert L.lbx_set_timeline(None) == 0
    a = tl.cpu().numpy()
    rt0, rt1 = a[:, 0].astype(np.float64), a[:, 1].astype(np.float64)
    st = a[:, NH:].reshape(waves, K, NP).astype(np.float64)
    ent, ext = a[:, 2].astype(np.float64), a[:, 3].astype(np.float64)
    life_rt = (rt1 - rt0) / 100.0  # us
    life_cy = st[:, K - 1, 2] - st[:, 0, 0]  # (stamp 4 is not taken in the last step)
    ghz = float(np.median(life_cy[life_rt > 0] / (life_rt[life_rt > 0] * 1e3)))
    inner = st[:, 1:K - 1, :]
    nxt = st[:, 2:K, 0]  # next step start
    d = {"apply": inner[:, :, 1] - inner[:, :, 0], "reset_path": inner[:, :, 2] - inner[:, :, 1],
         "prep_to_stores": inner[:, :, 3] - inner[:, :, 2], "stores_issue": inner[:, :, 4] - inner[:, :, 3],
         "wait_gathers": inner[:, :, 5] - inner[:, :, 4], "to_next_step": nxt - inner[:, :, 5]}
    tot = nxt - inner[:, :, 0]
    out.update({"clock_ghz_est": round(ghz, 3), "wave_life_us_mean": round(float(life_rt.mean()), 1),
                "step_cycles_mean": round(float(tot.mean())), "step_us_mean": round(float(tot.mean()) / ghz / 1e3, 2)})
    out["intervals_cycles_mean"] = {k: round(float(v.mean())) for k, v in d.items()}
    out["intervals_cycles_p90"] = {k: round(float(np.quantile(v, 0.9))) for k, v in d.items()}
    first = st[:, 0, :]
    out["first_step_cycles"] = round(float((st[:, 1, 0] - first[:, 0]).mean()))
    # realtime stamps (100 MHz): kernel entry, loop start, loop end, exit (write-back issued)
    t00 = ent.min()
    q = lambda x: [round(float(np.quantile(x, f)), 1) for f in (0.1, 0.5, 0.9, 1.0)]
    rec, img = a[:, 4].astype(np.float64), a[:, 5].astype(np.float64)
    out["prologue_us_q10_50_90_max"] = q((rt0 - ent) / 100.0)
    out["pro_records_us_q10_50_90_max"] = q((rec - ent) / 100.0)
    out["pro_image_us_q10_50_90_max"] = q((img - rec) / 100.0)
    out["pro_first_prep_us_q10_50_90_max"] = q((rt0 - img) / 100.0)
    out["epilogue_us_q10_50_90_max"] = q((ext - rt1) / 100.0)
    out["loop_us_q10_50_90_max"] = q((rt1 - rt0) / 100.0)
    out["entry_after_first_us_q10_50_90_max"] = q((ent - t00) / 100.0)
    out["exit_before_last_us_q10_50_90_max"] = q((ext.max() - ext) / 100.0)
    out["span_us"] = round(float((ext.max() - t00) / 100.0), 1)
    # where the slow waves run: wave life (entry -> exit) by XCC, by SIMD, by shader engine
    hw, xcc = a[:, 6].astype(np.int64), a[:, 7].astype(np.int64) & 0xF
    life = (ext - ent) / 100.0
    simd, cu, se = (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 13) & 7
    by = lambda key, n: {int(i): [int((key == i).sum()), round(float(life[key == i].mean()), 1)] for i in range(n)
                         if (key == i).any()}
    out["life_by_xcc"] = by(xcc, 16)
    out["life_by_simd"] = by(simd, 4)
    out["life_by_se"] = by(se, 8)
    out["life_by_cu"] = by(cu, 16)
    cid = xcc * 1024 + se * 64 + cu * 4 + simd
    u, inv, cnt = np.unique(cid, return_inverse=True, return_counts=True)
    out["waves_per_simd_hist"] = {int(k): int(v) for k, v in zip(*np.unique(cnt, return_counts=True))}
    # per SIMD: its waves' mean life; spread of that over SIMDs, and within-SIMD spread
    ms = np.array([life[inv == i].mean() for i in range(len(u))])
    out["simd_mean_life_q10_50_90"] = [round(float(np.quantile(ms, f)), 1) for f in (0.1, 0.5, 0.9)]
    out["life_q10_50_90_max"] = q(life)
    order = np.argsort(ent)
    gens = []
    for g0 in range(0, waves, 4096):
        idx = order[g0:g0 + 4096]
        gens.append({"start_us": round(float((ent[idx].min() - t00) / 100.0), 1),
                     "end_us": round(float((ext[idx].max() - t00) / 100.0), 1),
                     "step_cycles": round(float(tot[idx].mean()))})
    out["generations"] = gens
    if args.save:
        np.savez_compressed(args.save, stamps=a)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
