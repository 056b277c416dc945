#!/usr/bin/env python3
"""Mismatch report of k_rollout_lean against K x (policy + step_device): which envs, rows,
columns and steps differ, for a few (B, config) cases.  Diagnostic only.

    python tools/lean_diag.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd"), os.path.join(REPO, "tests")]


def run(B, kw, kind="random", K=20, L=20):
    import torch
    from test_gpu_lean import _staggered_pair
    a_env, b_env = _staggered_pair(B, L, kw)
    kern = a_env.rollout_kernel(K)
    R = a_env.cfg.obs_rows
    obs = torch.empty((K, B, R, 8), device="cuda")
    rew = torch.empty((K, B), device="cuda")
    dn = torch.empty((K, B), dtype=torch.uint8, device="cuda")
    act = torch.empty((K, B), dtype=torch.int32, device="cuda")
    a_env.rollout(kind, K, obs_out=obs, reward_out=rew, done_out=dn, actions_out=act)
    first = None
    for k in range(K):
        ak = b_env.policy(kind)
        b_env.step_device(ak)
        bad_a = (act[k] != ak)
        bad_o = (obs[k] != b_env.obs) & ~(torch.isnan(obs[k]) & torch.isnan(b_env.obs))
        bad_r = rew[k] != b_env.rewards
        bad_d = dn[k] != b_env.dones
        env_bad = bad_o.any(dim=(1, 2)) | bad_r | bad_d | bad_a
        n = int(env_bad.sum())
        if n:
            idx = torch.nonzero(env_bad).flatten()
            rows = torch.nonzero(bad_o.any(dim=0).any(dim=1)).flatten().tolist()
            cols = torch.nonzero(bad_o.any(dim=0).any(dim=0)).flatten().tolist()
            print(f"  step {k}: {n} envs bad (act {int(bad_a.sum())} obs {int(bad_o.any(dim=(1, 2)).sum())} "
                  f"rew {int(bad_r.sum())} done {int(bad_d.sum())}); rows {rows} cols {cols}; "
                  f"first envs {idx[:8].tolist()} lane {(idx[:8] % 64).tolist()} wave {(idx[:8] // 64).tolist()}")
            if first is None:
                first = k
                P = 2 * R
                bi = torch.nonzero(bad_o).cpu().numpy()  # (env, row, col)
                import collections
                el = bi[:, 0] % 64
                q = el * R + bi[:, 1]  # row-per-lane copy-out: row q by lane q % 64, round q // 64
                sl, it = q % 64, q // 64
                print("   half", collections.Counter((bi[:, 2] >= 4).tolist()))
                print("   bad cols", collections.Counter(bi[:, 2].tolist()))
                print("   storing lane", sorted(collections.Counter(sl.tolist()).items())[:40])
                print("   store instr", sorted(collections.Counter(it.tolist()).items()))
                print("   env lane", sorted(collections.Counter(el.tolist()).items())[:40])
                print("   row", sorted(collections.Counter(bi[:, 1].tolist()).items()))
                blk = bi[:, 0] // 256
                print("   blocks", len(set(blk.tolist())), "min", blk.min(), "max", blk.max(),
                      "wave in block", collections.Counter(((bi[:, 0] // 64) % 4).tolist()))
                dd = dn[k].bool()
                print("   done envs in bad waves:", int(dd.view(-1, 64)[torch.unique(torch.from_numpy(bi[:, 0] // 64)).cuda()].sum()),
                      "of", len(set((bi[:, 0] // 64).tolist())), "waves")
                e = int(idx[0])
                print("   lean obs", obs[k, e].cpu().numpy().round(4).tolist())
                print("   step obs", b_env.obs[e].cpu().numpy().round(4).tolist())
                print("   rew", float(rew[k, e]), float(b_env.rewards[e]), "done", int(dn[k, e]), int(b_env.dones[e]),
                      "act", int(act[k, e]), int(ak[e]))
                steps = b_env.stats()[e].cpu().numpy()
                print("   step-env stats row", steps.round(4).tolist())
            if k > first + 3:
                break
    print(f"B={B} kw={kw} kind={kind} K={K} L={L} kernel={kern}: {'OK' if first is None else 'first bad step %d' % first}")


if __name__ == "__main__":
    lib = os.environ.get("LEAN_LIB")
    if lib:
        from lbk8s import _native
        _native.LIB_PATH = os.path.abspath(lib)
    run(65600, {})
    run(131072, {}, K=1, L=20)
    run(131072, dict(reward_function="latency"))
    run(65600, dict(reward_function="multi"))
    run(131072, {}, K=2, L=20)
    run(262144, {})
    run(131072, {}, kind="endpoint_cpu")
