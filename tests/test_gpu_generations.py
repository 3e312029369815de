"""The generation controllers (pongmi.generations) on small configurations, with the thresholds forced
so each branch of the reference's loop runs: promotion (checkpoint written with the reference's keys
in its order, modelA <- modelB, RNN: the promoted net joins the runtime pool and the next generation
restarts B from A), fault after max_retries (fault checkpoint, modelB reset), and the RNN resume
from the latest-state checkpoint (parameters, Adam moments, counters restored; pool read from the
checkpoint directory without fault files). Every checkpoint loads with weights_only=True into the
reference's modules and optimizers (train_iterative.py:212-297, train_rnn_iterative.py:225-885)."""
import random

import pytest
import torch

pytestmark = pytest.mark.gpu

ENV = dict(render_size=400, paddle_width=0.2, paddle_speed=0.03, max_score=3, enable_render=False, enable_spin=True,
           magnus_factor=0.025, restitution=1, friction=0.6, ball_mass=1.0, world_ball_radius=0.03,
           ball_speed_range=[0.03, 0.05], spin_range=[-5, 5], ball_angle_intervals=[[-60, -30], [30, 60]],
           speed_scale_every=1, speed_increment=0.1)
QNET_KEYS = ["modelB", "optimizer", "epsilon", "episode", "modelA"]
RNN_OK_KEYS = ["modelA_state", "modelB_state", "optimizer_B_state", "epsilon", "episode", "generation",
               "train_steps_count", "old_state_for_reset"]
RNN_FAULT_KEYS = ["modelB_state", "optimizer_B_state", "epsilon", "episode", "generation", "modelA_state",
                  "train_steps_count", "old_state_for_reset"]
RNN_LATEST_KEYS = ["modelA_state", "modelB_state", "optimizer_B_state", "epsilon", "global_episode_count",
                   "current_generation_active", "done_generations_count", "train_steps_count", "old_state_for_reset"]


def _equal_sd(a, b):
    return list(a) == list(b) and all(torch.equal(a[k].cpu(), b[k].cpu()) for k in a)


# ---------------------------------------------------------------------------------------- QNet
def _qnet_cfg(tmp_path, **kw):
    from models.qnet import QNet
    torch.manual_seed(5)
    d = tmp_path / "checkpoints"
    d.mkdir()
    init = QNet(7, 3).state_dict()
    torch.save({"modelB": init, "epsilon": 0.5, "episode": 7}, d / "model4-12.pth")
    torch.manual_seed(6)
    torch.save({"modelB": QNet(7, 3).state_dict()}, d / "model4-3.pth")
    t = dict(max_generations=2, episodes_per_generation=300, eval_episodes=24, max_retries_for_generation=2,
             win_rate_interval=100, target_update_interval=50, model_id=9, opponent_pool_ratio=0.33,
             curr_win_threshold=0.0, pool_win_threshold=0.0, lr=2.5e-4, gamma=0.99, batch_size=64,
             memory_size=1 << 16, epsilon_decay=0.995, min_epsilon=0.02, init_model_path=str(d / "model4-12.pth"))
    t.update(kw)
    return {"env": ENV, "training": t}, d, init


def _check_qnet_ckpt(path):
    from models.qnet import QNet
    cp = torch.load(path, map_location="cpu", weights_only=True)
    assert list(cp) == QNET_KEYS
    net = QNet(7, 3)
    net.load_state_dict(cp["modelB"], strict=True)
    heads = list(net.fc_V.parameters()) + list(net.fc_A.parameters())
    torch.optim.Adam(heads, lr=2.5e-4).load_state_dict(cp["optimizer"])  # train_iterative.py:101-104
    return cp


def test_qnet_generations_promote(tmp_path):
    from pongmi.generations import QNetGenerations
    cfg, d, init = _qnet_cfg(tmp_path)
    lines = []
    G = QNetGenerations(cfg, n_arenas=512, seed=1, log=lines.append)
    assert len(G.pool) == 2 and G.L.counters()["episodes"] == 7 and G.L.updates_per_step == 512
    G.run(rng=random.Random(0))
    assert G.done_generations == 2
    for gen in (1, 2):
        cp = _check_qnet_ckpt(d / f"model9-{gen}.pth")
        assert _equal_sd(cp["modelA"], cp["modelB"])  # modelA <- modelB before saving (:264-266)
        assert cp["episode"] >= 7 + 300 * gen and 0.02 <= cp["epsilon"] < 0.5
    assert not _equal_sd(torch.load(d / "model9-2.pth", weights_only=True)["modelB"], init)
    assert any(s.startswith("[Gen 1] vs A:") for s in lines) and "升級! generation 2 done." in lines
    assert "[Saved] model9-2.pth" in lines and any(s.startswith("[Ep ") and ", interval:" in s for s in lines)


def test_qnet_generations_fault_resets_b(tmp_path):
    from pongmi.generations import QNetGenerations
    cfg, d, init = _qnet_cfg(tmp_path, max_generations=1, curr_win_threshold=1.1, episodes_per_generation=150)
    lines = []
    G = QNetGenerations(cfg, n_arenas=512, seed=2, log=lines.append)
    G.run(rng=random.Random(1))
    assert lines.count("未達标，继续尝试…") == 1 and "[Fault] model9-1_fault.pth" in lines
    cp = _check_qnet_ckpt(d / "model9-1_fault.pth")
    assert cp["optimizer"]["state"][0]["step"] > 0
    c = G.L.counters()
    assert c["epsilon"] == 1.0 and c["train_steps"] == 0 and c["size"] == 0  # reset_B (:213-224)
    got = G.L.modelB_state_dict()
    assert all(torch.equal(got[k].cpu(), init[k]) for k in init if "epsilon" not in k)


def test_qnet_generations_replay_ratio(tmp_path):
    """The reference trains once per env step: a try of E episodes runs ~E x mean episode length
    updates and its target network (interval 1000) syncs within the try. The controller's default
    (replay_ratio 1: U = n updates per vector step) keeps that: train_steps per try equals the env
    steps the try played, and the target follows modelB at the sync points."""
    from pongmi.generations import QNetGenerations, _Progress, _play_episodes
    cfg, d, init = _qnet_cfg(tmp_path, max_generations=1, episodes_per_generation=400, target_update_interval=1000,
                             batch_size=256)
    G = QNetGenerations(cfg, n_arenas=512, seed=4, log=lambda *_: None)
    L = G.L
    c0 = L.counters()
    c = _play_episodes(L, 400, _Progress(L, 100, "qnet", lambda *_: None), G.check_every)
    env_steps = (c["step"] - c0["step"]) * L.n
    eps = c["episodes"] - c0["episodes"]
    assert c["train_steps"] == env_steps  # one update per pushed transition
    assert eps >= 400 and 15 * eps <= c["train_steps"] <= 120 * eps  # ~mean episode length (~38) per episode
    assert c["train_steps"] >= 1000
    from pongmi.qnet import pack_state_dict
    p0 = pack_state_dict(G.old_state, "cpu")
    assert not torch.equal(L.paramsT.cpu()[4672:5192], p0[4672:5192])  # the target synced with a trained modelB
    assert c["max_prio"] == float(L.prios.max())  # U * batch >= n: the commit keeps the array maximum


# ---------------------------------------------------------------------------------------- QNetRNN
def _rnn_cfg(tmp_path, **kw):
    d = tmp_path / "checkpoints_rnn"
    t = dict(trace_length=8, max_generations=2, episodes_per_generation=300, eval_episodes=16,
             max_retries_for_generation=2, curr_win_threshold=0.0, pool_win_threshold=0.0, lr=1e-4, gamma=0.99,
             batch_size=32, memory_size=40000, min_episodes_for_training_start=2,
             initial_epsilon_per_generation=0.7, epsilon_decay=0.999, min_epsilon=0.05, target_update_interval=100,
             model_id_prefix="rnn_t_", init_model_path_rnn=None, ckpt_dir_rnn=str(d), opponent_pool_ratio=0.4,
             win_rate_interval=100, save_latest_checkpoint_interval_steps=300,
             latest_checkpoint_filename="latest_rnn_training_state.pth")
    t.update(kw)
    return {"env": {**ENV, "speed_scale_every": 5, "speed_increment": 0.2}, "training": t}, d


def _check_rnn_ckpt(path, keys):
    from models.qnet_rnn import QNetRNN
    cp = torch.load(path, map_location="cpu", weights_only=True)
    assert list(cp) == keys
    net = QNetRNN(7, 3)
    net.load_state_dict(cp["modelB_state"], strict=True)
    torch.optim.Adam(net.parameters(), lr=1e-4).load_state_dict(cp["optimizer_B_state"])
    QNetRNN(7, 3).load_state_dict(cp["old_state_for_reset"], strict=True)
    return cp


def test_rnn_generations_promote_pool_and_resume(tmp_path):
    from pongmi import checkpoint
    from pongmi.drqn import PARAM_SHAPES
    from pongmi.generations import RNNGenerations
    cfg, d = _rnn_cfg(tmp_path)
    lines = []
    G = RNNGenerations(cfg, n_arenas=128, seed=3, log=lines.append)
    assert G.L.updates_per_step == 128  # replay ratio 1: one DRQN update per env step
    assert G.L.n_pool == 0 and "[WARNING] Opponent pool is empty! ModelB will only train against ModelA." in lines
    G.run(rng=random.Random(2))
    assert G.done_generations == 2 and G.L.n_pool == 2  # promoted nets join the runtime pool (:855-859)
    assert any("Epsilon reset to 0.7" in s for s in lines)
    for gen in (1, 2):
        cp = _check_rnn_ckpt(d / f"rnn_t_{gen}.pth", RNN_OK_KEYS)
        assert cp["generation"] == gen and cp["train_steps_count"] > 0
        assert _equal_sd(cp["modelA_state"], cp["modelB_state"]) and _equal_sd(cp["old_state_for_reset"], cp["modelA_state"])
    # gen 2's redraws pick the promoted nets (slots 1..n_pool); few of the episodes in flight finish
    # within a 300-episode budget, so count the draws rather than the finished episodes
    assert int((G.L.opp > 0).sum()) > 0 and int(G.L.opp.max()) <= 2
    latest = _check_rnn_ckpt(d / "latest_rnn_training_state.pth", RNN_LATEST_KEYS)
    # saved right after update k * 300, recording k * 300 - 1 as the reference does (:519-528)
    assert latest["train_steps_count"] % 300 == 299

    # resume: B, A, Adam, epsilon, counters from the latest checkpoint; pool = every non-fault .pth
    torch.save({"modelB_state": latest["modelB_state"]}, d / "rnn_t_3_fault.pth")
    lines2 = []
    G2 = RNNGenerations(cfg, n_arenas=128, seed=4, log=lines2.append)
    assert any(s.startswith("[INFO] Resumed from latest checkpoint.") for s in lines2)
    assert G2.L.n_pool == 3 and not any("fault" in s for s in lines2 if "Loaded RNN pool model" in s)
    assert _equal_sd(G2.L.modelB_state_dict(), latest["modelB_state"])
    assert _equal_sd(G2.L.modelA_state_dict(), latest["modelA_state"])
    c = G2.L.counters()
    assert c["episodes"] == latest["global_episode_count"] and abs(c["epsilon"] - latest["epsilon"]) < 1e-12
    assert c["train_steps"] == latest["train_steps_count"]
    m, v, step = checkpoint.adam_moments(G2.L.learner.optimizer_state_dict(), PARAM_SHAPES)
    m0, v0, step0 = checkpoint.adam_moments(latest["optimizer_B_state"], PARAM_SHAPES)
    assert step == step0 and torch.equal(m, m0) and torch.equal(v, v0)
    assert G2.done_generations == 0 and G2.current_generation == 0  # reset before the loop (:625-626)


def test_rnn_generations_fault_resets_b(tmp_path):
    from pongmi.generations import RNNGenerations
    cfg, d = _rnn_cfg(tmp_path, max_generations=1, max_retries_for_generation=1, curr_win_threshold=1.1,
                      episodes_per_generation=200, save_latest_checkpoint_interval_steps=0)
    lines = []
    G = RNNGenerations(cfg, n_arenas=128, seed=5, log=lines.append)
    G.run(rng=random.Random(3))
    cp = _check_rnn_ckpt(d / "rnn_t_1_fault.pth", RNN_FAULT_KEYS)
    assert cp["train_steps_count"] > 0 and not (d / "latest_rnn_training_state.pth").exists()
    assert "[INFO] modelB reset to current modelA's state." in lines
    c = G.L.counters()
    assert c["epsilon"] == 1.0 and c["train_steps"] == 0
    assert _equal_sd(G.L.modelB_state_dict(), G.L.modelA_state_dict())
    assert G.L.learner.optimizer_state_dict()["state"] == {}


def test_training_scripts_read_config_from_cwd(tmp_path):
    """scripts/train_iterative.py / train_rnn_iterative.py as a user runs them: config file in the
    working directory, checkpoints where the config points (a child process, one at a time)."""
    import os
    import subprocess
    import sys

    import yaml
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    scripts = os.path.join(root, "pingpong-selfplay-ai_amd", "scripts")
    qcfg, d, _ = _qnet_cfg(tmp_path, max_generations=1, episodes_per_generation=100)
    qcfg["training"]["init_model_path"] = "checkpoints/model4-12.pth"  # relative to the CWD, as in config.yaml
    rcfg, rd = _rnn_cfg(tmp_path, max_generations=1, episodes_per_generation=100)
    qcfg["training"]["batch_size"] = 64
    rcfg["training"]["ckpt_dir_rnn"] = "checkpoints_rnn"
    (tmp_path / "config.yaml").write_text(yaml.safe_dump(qcfg))
    (tmp_path / "config_rnn.yaml").write_text(yaml.safe_dump(rcfg))
    for script, made in (("train_iterative.py", d / "model9-1.pth"), ("train_rnn_iterative.py", rd / "rnn_t_1.pth")):
        out = subprocess.run([sys.executable, os.path.join(scripts, script), "--arenas", "256"], cwd=tmp_path,
                             capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr[-2000:]
        assert made.exists(), out.stdout[-2000:]
    assert "=== RNN Training: Generation 1/1 ===" in out.stdout


def test_rnn_generations_replay_ratio_and_exact_saves(tmp_path):
    """RNN controller at its defaults (64 arenas, one DRQN update per env step): train steps follow
    the env steps once training is enabled, the target syncs (interval 100 here), and every
    latest-state save lands exactly after update k * interval with k * interval - 1 recorded."""
    from pongmi.generations import RNNGenerations, _Progress, _play_episodes
    cfg, d = _rnn_cfg(tmp_path, max_generations=1, episodes_per_generation=150, save_latest_checkpoint_interval_steps=700)
    saves = []
    G = RNNGenerations(cfg, seed=6, log=lambda *_: None)
    assert G.L.n == 64 and G.L.updates_per_step == 64
    orig = G.save_latest
    G.save_latest = lambda train_steps=None: (saves.append((train_steps, G.L.learner.stats()["steps"])),
                                              orig(train_steps))
    L = G.L
    target0 = L.learner.target.cpu().clone()
    c = _play_episodes(L, 150, _Progress(L, 100, "rnn", lambda *_: None), G.check_every, G._on_check, G._step)
    st = L.learner.stats()["steps"]
    assert st % 64 == 0 and st >= 150 * 10 and st <= c["step"] * 64
    assert saves and all(ts == after - 1 and after % 700 == 0 for ts, after in saves)
    assert len(saves) == st // 700
    assert not torch.equal(L.learner.target.cpu(), target0)  # synced every 100 updates (interval)
    assert c["status"] == 0
