"""The inference rollout megakernel (K9, pm_rollout / pongmi.rollout): configs[1] in one launch.

`steps` vector steps of the launch must equal, bit for bit, the stepped composition it replaces —
per vector step c: modelB's heads refolded with fresh noise (qnet.fold FRESH, Philox(seed_net, c)),
both players' act (qnet.act: A greedy, B eps-greedy with Philox(seed_env, c)), one K1 env step with
autoreset (step-keyed serves) — itself pinned to the reference by test_gpu_qnet_replay.py (act
against the f32 oracle), test_gpu_env.py (the tick and the serves) and test_gpu_selfplay.py. Checked:
the fp64 state, scores, bounces and observations after the launch, the episode / point counters,
ragged arena counts (not multiples of the 32-arena tile), launches that chain (counter continuity),
the epsilon extremes, and the failure paths.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _models(seed):
    from models.qnet import QNet
    from pongmi import _lib
    from pongmi.qnet import fold, pack_state_dict
    torch.manual_seed(seed)
    mA, mB = QNet(7, 3), QNet(7, 3)
    wA = fold(pack_state_dict(mA.state_dict()), _lib.PM_FOLD_TRAIN).reshape(-1)
    return wA, pack_state_dict(mB.state_dict()).reshape(-1)


def _env(n, seed):
    from pongmi.env import PongEnv2PBatch
    env = PongEnv2PBatch(n, seed=seed, autoreset=True)
    env.reset()
    return env


def _stepped(env, wA, paramsB, eps, seed_net, steps):
    from pongmi import _lib
    from pongmi.qnet import act, fold
    tot = np.zeros(4, np.int64)
    for _ in range(steps):
        c = env.counter
        wB = fold(paramsB, _lib.PM_FOLD_TRAIN_FRESH, seed=seed_net, counter=c)
        aA, aB = act(wA.reshape(1, -1), None, wB, env.obsA, env.obsB, eps, seed=env.seed, counter=c)[:2]
        _, (rA, rB), done, _ = env.step(aA, aB)
        d = done.bool()
        tot += np.array([int(d.sum()), int((d & (rB > 0)).sum()), int((rA > 0).sum()), int((rB > 0).sum())])
    return tot


def _same_env(a, b):
    sa, sb = a.get_state(), b.get_state()
    for k in ("x", "y", "vx", "vy", "spin", "top", "bot", "scoreA", "scoreB", "bounces"):
        assert np.array_equal(sa[k], sb[k]), k
    assert torch.equal(a.obsA, b.obsA) and torch.equal(a.obsB, b.obsB)
    assert a.counter == b.counter


@pytest.mark.parametrize("n,steps,eps", [(1, 90, 0.02), (100, 120, 0.02), (4096, 150, 0.02), (333, 60, 1.0),
                                         (257, 60, 0.0)])
def test_rollout_equals_stepped(n, steps, eps):
    from pongmi.rollout import STATS, SelfPlayRollout
    wA, paramsB = _models(n)
    seed_env, seed_net = 0x5EED + n, 77 + n
    fused, ref = _env(n, seed_env), _env(n, seed_env)
    st = SelfPlayRollout(fused, wA, paramsB, epsilon=eps, seed_net=seed_net).run(steps)
    tot = _stepped(ref, wA, paramsB, eps, seed_net, steps)
    _same_env(fused, ref)
    assert [st[k] for k in STATS] == tot.tolist()
    assert st["episodes"] > 0 and st["points_A"] + st["points_B"] >= 2 * st["episodes"]


def test_rollout_launches_chain():
    """Two launches of 40 + 75 steps equal one of 115 (the heads workspace and the Philox counters
    continue from env.counter), and equal the stepped path after an interleaved stepped stretch."""
    from pongmi.rollout import SelfPlayRollout
    n = 1000
    wA, paramsB = _models(5)
    a, b, c = _env(n, 9), _env(n, 9), _env(n, 9)
    ra, rb = SelfPlayRollout(a, wA, paramsB, seed_net=3), SelfPlayRollout(b, wA, paramsB, seed_net=3)
    s1, s2 = ra.run(40), ra.run(75)
    s = rb.run(115)
    _same_env(a, b)
    assert s["episodes"] == s1["episodes"] + s2["episodes"]
    _stepped(c, wA, paramsB, 0.02, 3, 20)
    SelfPlayRollout(c, wA, paramsB, seed_net=3).run(95)
    _same_env(a, c)


def test_rollout_failure_paths():
    from pongmi import _lib
    from pongmi.env import PongEnv2PBatch
    from pongmi.rollout import SelfPlayRollout
    wA, paramsB = _models(1)
    with pytest.raises(_lib.PongmiError):
        SelfPlayRollout(PongEnv2PBatch(8, autoreset=False), wA, paramsB)
    with pytest.raises(_lib.PongmiError):
        SelfPlayRollout(PongEnv2PBatch(2, autoreset=True, serve_table=np.zeros((2, 1, 3))), wA, paramsB)
    with pytest.raises(ValueError):
        SelfPlayRollout(_env(8, 1), wA[:-1], paramsB)
    env = _env(64, 2)
    before = env.get_state()
    r = SelfPlayRollout(env, wA, paramsB)
    assert r.run(0)["episodes"] == 0 and env.counter == 0
    after = env.get_state()
    assert all(np.array_equal(before[k], after[k]) for k in before)
    with pytest.raises(ValueError):
        r.run(-1)
