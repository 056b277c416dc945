"""Multi-rank learners on the GPU: 2 ranks, launched like the driver's
bench (torch.distributed.run on 127.0.0.1).  On a one-GPU box both ranks share the card
over gloo (LBK8S_DIST_BACKEND=gloo); the code path is the RCCL one minus the backend."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _env():
    env = dict(os.environ, LBK8S_DIST_BACKEND="gloo", PYTHONPATH=os.path.join(REPO, "gym-loadbalancing_amd"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("algo", ["ppo", "dqn"])
def test_two_ranks_graph_equals_eager(tmp_path, algo):
    """Averaged gradients keep the replicas identical, and the split-graph step (graphs
    around the gradient all_reduce: PPO's minibatch step, DQN's train step) computes the
    eager update."""
    from lbk8s.dist import free_port
    out = tmp_path / "res.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(REPO, "tests", "dist_ppo_worker.py"), str(out), algo]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["world"] == 2
    assert res["ranks_agree_graphs0"] and res["ranks_agree_graphs1"], res
    assert res["graph_eq_eager"], res
    assert res["returns_eq"], res


def test_cli_nproc_two_ranks(tmp_path):
    """python -m lbk8s.cli --nproc 2: two ranks train, rank 0 saves, each rank writes its
    VecMonitor file."""
    r = subprocess.run([sys.executable, "-m", "lbk8s.cli", "--alg", "ppo_deepsets", "--nproc", "2",
                        "--num_envs", "32", "--total_steps", str(32 * 100 * 2), "--num_endpoints", "8",
                        "--rejection"], cwd=tmp_path, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert any(ln.get("world_size") == 2 and "saved" in ln for ln in lines), r.stdout[-2000:]
    for rank in (0, 1):
        mon = tmp_path / f"vec_loadbalancer_k8s_gym_results_rank{rank}.monitor.csv"
        assert mon.exists()
        assert len(mon.read_text().splitlines()) == 2 + 32 * 2  # header lines + 2 episodes per env
    saved = [p for p in os.listdir(tmp_path) if p.startswith("ppo_deepsets_env_loadbalancer")]
    assert len(saved) == 1


def test_rccl_one_rank_multi_path_equals_single_rank(tmp_path):
    """The RCCL code path on a one-GPU box: one process forms a one-rank nccl (= RCCL)
    group and runs PPO and DQN with the multi-rank path forced (LBK8S_FORCE_MULTI=1:
    broadcast, gradient all_reduce between the split HIP graphs, episode-return all_reduce);
    the result equals the single-rank graph path's bit for bit."""
    out = tmp_path / "res.json"
    env = dict(os.environ, LBK8S_DIST_BACKEND="nccl", PYTHONPATH=os.path.join(REPO, "gym-loadbalancing_amd"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "dist_force_worker.py"), str(out)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(out.read_text())
    print(json.dumps(res))
    assert res["backend"] == "nccl" and res["world"] == 1
    for algo in ("ppo", "dqn"):
        assert res[algo]["equal"], res[algo]
        assert res[algo]["returns_multi"] == res[algo]["returns_single"], res[algo]
