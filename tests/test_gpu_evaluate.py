"""Batched evaluators (pongmi.evaluate) against the reference's sequential eval loops
(scripts/train_iterative.py:171-196).

1. The reference loop body, restated here, run episode by episode over the drop-in PongEnv2P and
   QNet modules with the same global `random` seed: identical per-episode outcomes and the same
   `random` stream consumption.
2. The oracle (C env + the float32 QNet restatement in the device's evaluation order) playing the
   same episodes: every episode's outcome and length are identical.
"""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ENV_KW = dict(paddle_width=0.2, paddle_speed=0.03, max_score=3, enable_spin=True, magnus_factor=0.025, restitution=1,
              friction=0.6, ball_mass=1.0, world_ball_radius=0.03, ball_speed_range=[0.03, 0.05], spin_range=[-5, 5],
              ball_angle_intervals=[[-60, -30], [30, 60]], speed_scale_every=1, speed_increment=0.1)


def _qnet(sd, train):
    from models.qnet import QNet
    net = QNet(7, 3).cuda()
    net.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()})
    net.train(train)
    return net


def _sd(g, who):
    return {k[len(who) + 1:]: v for k, v in g.items() if k.startswith(who + ".") and "q_" not in k}


def _random_sd(seed):
    from models.qnet import QNet
    torch.manual_seed(seed)
    return {k: v.clone().numpy() for k, v in QNet(7, 3).state_dict().items()}


def _ref_episode(env, A, B):
    """The body of eval_vs_model's / eval_vs_pool's episode loop (train_iterative.py:174-180)."""
    oA, oB = env.reset()
    done = False
    length = 0
    while not done:
        aA = A(torch.tensor(oA, dtype=torch.float32, device="cuda").unsqueeze(0)).argmax(1).item()
        aB = B(torch.tensor(oB, dtype=torch.float32, device="cuda").unsqueeze(0)).argmax(1).item()
        (nA, nB), (rA, rB), done, _ = env.step(aA, aB)
        oA, oB = nA, nB
        length += 1
    return rB > rA, length


def test_eval_vs_model_matches_reference_loop(golden):
    from envs.my_pong_env_2p import PongEnv2P
    from pongmi.evaluate import eval_vs_model
    g = golden("qnet")
    A, B = _qnet(_sd(g, "modelA"), True), _qnet(_sd(g, "modelB"), True)
    env = PongEnv2P(**ENV_KW)
    E = 24
    random.seed(1234)
    ref = [_ref_episode(env, A, B) for _ in range(E)]
    state_ref = random.getstate()
    random.seed(1234)
    rate, wins, length = eval_vs_model(env, A, B, E, return_details=True)
    assert random.getstate() == state_ref  # the same draws from the global stream
    assert wins.tolist() == [w for w, _ in ref]
    assert length.tolist() == [n for _, n in ref]
    assert rate == sum(w for w, _ in ref) / E


def test_eval_vs_pool_matches_reference_loop(golden):
    from envs.my_pong_env_2p import PongEnv2P
    from pongmi.evaluate import eval_vs_pool
    g = golden("qnet")
    B = _qnet(_sd(g, "modelB"), True)
    pool = [_qnet(_random_sd(100 + k), False) for k in range(3)]  # pool nets are in eval mode
    env = PongEnv2P(**ENV_KW)
    E = 24
    random.seed(99)
    ref = []
    for _ in range(E):
        opp = random.choice(pool)
        ref.append((pool.index(opp),) + _ref_episode(env, opp, B))
    state_ref = random.getstate()
    random.seed(99)
    rate, wins, length, opp = eval_vs_pool(env, B, pool, E, return_details=True)
    assert random.getstate() == state_ref
    assert opp.tolist() == [o for o, _, _ in ref]
    assert wins.tolist() == [w for _, w, _ in ref]
    assert length.tolist() == [n for _, _, n in ref]
    assert eval_vs_pool(env, B, [], 10) == 1.0


def test_eval_vs_model_against_oracle(golden, orc):
    """400 episodes against the oracle: the float32 QNet in the device's order (oracle.qnet_forward_f32,
    torch's float32 fold of mu + sigma*eps) + the C env stepping the same serves: every episode."""
    from pongmi.env import draw_serve, env_config
    from pongmi.evaluate import eval_vs_model
    g = golden("qnet")
    sdA, sdB = _sd(g, "modelA"), _sd(g, "modelB")
    E = 400
    rng = random.Random(7)
    rate, wins, length = eval_vs_model(dict(ENV_KW), _qnet(sdA, True), _qnet(sdB, True), E, rng=rng,
                                       return_details=True)
    cfg = env_config(**ENV_KW)
    rng = random.Random(7)
    serves = np.array([draw_serve(rng, cfg) for _ in range(E)])
    P = orc.make_params(orc.env_params_from_kwargs(**ENV_KW))
    arr = np.zeros(E, orc.ARENA_DTYPE)
    orc.serve_arenas(arr, np.ones(E, bool), serves[:, 0], serves[:, 1], serves[:, 2])
    wA = orc.fold_heads_f32(sdA, "train")  # train mode: mu + sigma * the nets' epsilon buffers
    wB = orc.fold_heads_f32(sdB, "train")
    oA, oB = orc.obs_of_arenas(arr)
    fin = np.zeros(E, bool)
    owin = np.zeros(E, bool)
    olen = np.zeros(E, np.int32)
    t = 0
    while not fin.all():
        aA = orc.argmax_first(orc.qnet_forward_f32(wA, oA))
        aB = orc.argmax_first(orc.qnet_forward_f32(wB, oB))
        oA, oB, rew, done = orc.step_arenas(P, arr, aA, aB)
        t += 1
        new = (done > 0) & ~fin
        owin |= new & (rew[:, 1] > rew[:, 0])
        olen[new] = t
        fin |= new
    assert np.array_equal(owin, wins) and np.array_equal(olen, length)
    assert rate == owin.mean()
