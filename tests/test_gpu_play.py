"""The match megakernel (K8, pm_play / pongmi.play): whole greedy episodes in one launch.

It must give, episode by episode, exactly what the stepped path gives (one act launch + one env
launch per tick, itself pinned to the reference's loops in test_gpu_evaluate.py and
test_gpu_tournament.py): final scores, lengths and the last tick's reward sign, for QNet nets
(folded eval / train weights), the ball follower, mixed pairs, ragged group sizes (not multiples of
the 128-arena block), and the serves the evaluators draw from `random`. The follower and the tick
are checked exactly against the oracle env; the failure paths (unfinished within max_steps, bad
net id) raise.
"""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ENV_KW = dict(paddle_width=0.2, paddle_speed=0.03, max_score=3, enable_spin=True, magnus_factor=0.025, restitution=1,
              friction=0.6, ball_mass=1.0, world_ball_radius=0.03, ball_speed_range=[0.03, 0.05], spin_range=[-5, 5],
              ball_angle_intervals=[[-60, -30], [30, 60]], speed_scale_every=1, speed_increment=0.1)


def _nets(k, seed=0):
    from models.qnet import QNet
    from pongmi.evaluate import folded_weights
    from pongmi import _lib
    out = []
    for i in range(k):
        torch.manual_seed(seed + i)
        m = QNet(7, 3)
        out.append(folded_weights((m.state_dict(), _lib.PM_FOLD_TRAIN if i % 2 else _lib.PM_FOLD_EVAL), "cuda"))
    return torch.stack(out)


def _serves(E, seed):
    from pongmi.env import draw_serve, env_config
    rng, cfg = random.Random(seed), env_config(**ENV_KW)
    return np.array([draw_serve(rng, cfg) for _ in range(E)], np.float64)


@pytest.mark.parametrize("E,n_opp", [(1, 1), (1000, 1), (3001, 5)])
def test_play_matches_stepped_episodes(E, n_opp):
    from pongmi.evaluate import run_episodes, run_episodes_stepped
    w = _nets(n_opp + 1, seed=E)
    opp = None if n_opp == 1 else np.random.default_rng(E).integers(0, n_opp, E).astype(np.int32)
    serves = _serves(E, E)
    wins, length = run_episodes(ENV_KW, w[:n_opp], opp, w[n_opp], serves)
    wins_s, length_s = run_episodes_stepped(ENV_KW, w[:n_opp], opp, w[n_opp], serves)
    assert np.array_equal(length, length_s) and np.array_equal(wins, wins_s)
    assert (length > 0).all()


@pytest.mark.parametrize("per_block", [128, 640, 1024])
def test_play_lane_refill_matches_stepped(per_block):
    """Blocks with more slots than columns: finished columns take the next slot of the range (1, 5
    and 8 slots per column). Every episode must equal the stepped loop's."""
    from pongmi.evaluate import run_episodes_stepped
    from pongmi.play import play
    E, n_opp = 8192, 3
    w = _nets(n_opp + 1, seed=77)
    opp = np.random.default_rng(1).integers(0, n_opp, E).astype(np.int32)
    serves = _serves(E, 21)
    sA, sB, length, last = play(ENV_KW, w, opp, np.full(E, n_opp), serves, per_block=per_block)
    wins_s, length_s = run_episodes_stepped(ENV_KW, w[:n_opp], opp, w[n_opp], serves)
    assert np.array_equal(length, length_s) and np.array_equal(last > 0, wins_s)
    assert (np.maximum(sA, sB) == 3).all()


def test_play_scores_and_follower_pairs_match_stepped():
    """Tournament shapes: QNet-QNet, QNet-follower, follower-QNet, follower-follower pairs, ragged."""
    from models.qnet import QNet
    from pongmi.tournament import _play_fused, _play_stepped
    models = {}
    for i in range(3):
        torch.manual_seed(40 + i)
        models[f"q{i}"] = (QNet(7, 3).eval().cuda(), "QNet")
    models["bot"] = ("HardcodedAgent", "HardcodedBallFollower")
    models["bot2"] = ("HardcodedAgent", "HardcodedBallFollower")
    plan = [("q0", "q1", 77), ("q2", "bot", 130), ("bot", "q0", 5), ("bot", "bot2", 64), ("q1", "q0", 200)]
    eps = [(a, b) for a, b, e in plan for _ in range(e)]
    serves = _serves(len(eps), 9)
    got = _play_fused(ENV_KW, models, eps, serves, "cuda", 1_000_000)
    ref = _play_stepped(ENV_KW, models, eps, serves, "cuda", 1_000_000)
    assert np.array_equal(got, ref)
    assert (got.max(1) == 3).all()


def test_play_follower_against_oracle(orc):
    """Ball follower vs ball follower, exact against the oracle env (no net: the in-kernel follower
    and tick alone). The QNet players are pinned to the oracle through eval_vs_model
    (test_gpu_evaluate.py), which runs on this kernel."""
    from pongmi.play import FOLLOWER, play
    E = 300
    serves = _serves(E, 11)
    sA, sB, length, last = play(ENV_KW, None, np.full(E, FOLLOWER), np.full(E, FOLLOWER), serves)
    P = orc.make_params(orc.env_params_from_kwargs(**ENV_KW))
    arr = np.zeros(E, orc.ARENA_DTYPE)
    orc.serve_arenas(arr, np.ones(E, bool), serves[:, 0], serves[:, 1], serves[:, 2])
    oA, oB = orc.obs_of_arenas(arr)
    fin = np.zeros(E, bool)
    olen = np.zeros(E, np.int32)
    olast = np.zeros(E, np.int8)
    score = np.zeros((E, 2), np.int64)
    tol = np.float32(0.01)
    follow = lambda o: np.where(o[:, 0] < o[:, 4] - tol, 0, np.where(o[:, 0] > o[:, 4] + tol, 2, 1))  # noqa: E731
    t = 0
    while not fin.all() and t < 100000:
        oA, oB, rew, done = orc.step_arenas(P, arr, follow(oA), follow(oB))
        t += 1
        new = (done > 0) & ~fin
        olen[new] = t
        olast[new] = np.sign(rew[new, 1] - rew[new, 0]).astype(np.int8)
        score[new, 0], score[new, 1] = arr["scoreA"][new], arr["scoreB"][new]
        fin |= new
    assert fin.all()
    assert np.array_equal(length, olen) and np.array_equal(last, olast)
    assert np.array_equal(sA, score[:, 0]) and np.array_equal(sB, score[:, 1])


def test_play_failure_paths():
    from pongmi.play import play
    w = _nets(1)
    serves = _serves(10, 1)
    with pytest.raises(RuntimeError, match="did not finish"):
        play(ENV_KW, w, np.zeros(10), np.zeros(10), serves, max_steps=3)
    with pytest.raises(ValueError):
        play(ENV_KW, w, np.zeros(10), np.full(10, 1), serves)
    sA, sB, length, last = play(ENV_KW, None, np.full(4, -1), np.full(4, -1), _serves(4, 2))
    assert (np.maximum(sA, sB) == 3).all() and (length > 0).all()
    assert play(ENV_KW, w, [], [], np.zeros((0, 3)))[0].shape == (0,)
