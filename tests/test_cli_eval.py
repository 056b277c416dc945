"""§8(f) rows 2-3: the run.py CLI equivalent (lbk8s.cli) and the run_test_deepset
evaluation loop (lbk8s.evaluate)."""
import numpy as np
import pytest
import torch


def test_cli_defaults_match_reference():
    from lbk8s.cli import build_parser, env_kwargs, model_name
    a = build_parser().parse_args([])
    # run.py:24-45
    assert a.alg == "dqn_deepsets" and a.env_name == "loadbalancer"
    assert int(a.num_endpoints) == 6 and a.rejection is False and int(a.num_zones) == 4
    assert int(a.num_nodes) == 24 and a.reward == "multi"
    assert a.training is True and a.testing is False and a.loading is False
    assert int(a.steps) == 200000 and int(a.total_steps) == 200000
    # run.py:189-191
    assert model_name("dqn_deepsets", "loadbalancer", 6, 4, "multi", 200000) == \
        "dqn_deepsets_env_loadbalancer_num_endpoints_6_num_zones_4_reward_multi_totalSteps_200000"
    # run.py:97-107
    kw = env_kwargs(False, 6, 4, 24, "multi")
    assert kw["latency_weight"] == 1.0 and kw["cpu_weight"] == 0 and kw["gini_weight"] == 0.0
    assert kw["arrival_rate_r"] == 100 and kw["call_duration_r"] == 1 and kw["episode_length"] == 100


def test_cli_rejects_sb3_algorithms():
    from lbk8s.cli import get_model
    for alg in ("ppo", "a2c", "recurrent_ppo", "mask_ppo", "bogus"):
        with pytest.raises(SystemExit):
            get_model(alg, None)


def test_monitor_csv_layout(tmp_path):
    from lbk8s.evaluate import write_monitor_csv
    res = {"r": np.array([3.0, -1.0]), "l": np.array([100, 100]), "wall_s": 0.5,
           "gini": np.array([0.1, 0.2])}
    path = tmp_path / "m.monitor.csv"
    write_monitor_csv(path, res, ("gini",))
    lines = path.read_text().splitlines()
    assert lines[0].startswith("#{") and lines[1] == "r,l,t,gini" and lines[2].startswith("3.0,100,")


@pytest.mark.gpu
def test_run_test_matches_single_episode_replay():
    """Episodes played side by side == each episode played alone (global env id i)."""
    from lbk8s import LBVecEnv
    from lbk8s.deepsets import DeepSetAgent, DQNDeepSetAgent
    from lbk8s.evaluate import TEST_ENV, greedy_actions, run_test
    from lbk8s.info import ST_RETURN
    torch.manual_seed(0)
    for agent in (DeepSetAgent(8).cuda(), DQNDeepSetAgent(8).cuda()):
        res = run_test(agent, n_episodes=64, seed=5, episode_length=20)
        assert res["r"].shape == (64,) and (res["l"] == 20).all()
        kw = dict(TEST_ENV, episode_length=20)
        for i in (0, 37):
            env = LBVecEnv(1, seed=5, env_id_offset=i, auto_reset=False, as_tensors=True, **kw)
            obs = env.reset()
            for _ in range(20):
                obs, _, _, _ = env.step(greedy_actions(agent, obs, env.action_masks()))
            # the float64 episode return (the per-step rewards come back as float32)
            assert float(env.stats()[0, ST_RETURN]) == res["r"][i]


@pytest.mark.gpu
def test_cli_train_save_and_test(tmp_path, monkeypatch):
    from lbk8s import cli
    monkeypatch.chdir(tmp_path)
    r = cli.main(["--alg", "ppo_deepsets", "--total_steps", "1600", "--num_envs", "16"])
    assert (tmp_path / r["saved"]).exists()
    r2 = cli.main(["--alg", "ppo_deepsets", "--no_training", "--testing", "--test_path",
                   str(tmp_path / r["saved"]), "--test_episodes", "8"])
    assert len(r2["test_returns"]) == 8 and all(np.isfinite(r2["test_returns"]))
    r3 = cli.main(["--alg", "dqn_deepsets", "--total_steps", "120", "--num_envs", "16", "--testing",
                   "--test_path", "dqn_deepsets_env_loadbalancer_num_endpoints_6_num_zones_4_reward_multi_totalSteps_120"])
    assert len(r3["test_returns"]) == 1
