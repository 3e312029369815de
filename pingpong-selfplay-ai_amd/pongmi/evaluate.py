"""Batched evaluators: eval_vs_model / eval_vs_pool (scripts/train_iterative.py:171-196).

The reference plays `episodes` greedy episodes one after another on one PongEnv2P: each episode
is one env.reset() (its serve drawn from the global `random` stream, envs/my_pong_env_2p.py:94-110;
eval_vs_pool draws `random.choice(pool)` first) followed by ticks until a score reaches max_score
(a point does not re-serve). A win is rB > rA on the episode's LAST step (:180).

Here every episode is an arena of one PongEnv2PBatch, all advanced in lockstep (K1 + the fused
two-player act K2, both players greedy): the host draws the per-episode opponent and serve from
the same `random` stream in the reference's order, so episode e sees exactly the serve and the
opponent the reference's e-th episode would. The episodes run inside the match megakernel (K8,
pongmi.play): one launch plays every episode to the end with the arenas in registers. The nets act as their modules would: a QNet in
train mode uses mu + sigma * (its current epsilon buffers), in eval mode mu (models/qnet.py:43-50).
"""
import random as _pyrandom

import numpy as np
import torch

from . import _lib
from .env import PongEnv2PBatch, draw_serve, env_config
from .qnet import act as qnet_act
from .qnet import fold, pack_state_dict


def env_kwargs(env):
    """PongEnv2P constructor kwargs of `env` (the drop-in PongEnv2P, a PongEnv2PBatch, or a dict)."""
    if isinstance(env, dict):
        return dict(env)
    cfg = getattr(env, "_cfg", None)
    if cfg is None:
        cfg = getattr(env, "cfg", None)
    if cfg is None:
        raise TypeError("env must be a PongEnv2P, a PongEnv2PBatch or a dict of PongEnv2P kwargs")
    return dict(cfg)


def folded_weights(net, device):
    """Effective weights [PM_QNET_NW] of a QNet module (mode as its forward would use it) or of a
    (state_dict, fold_mode) pair."""
    if isinstance(net, tuple):
        sd, mode = net
        block = pack_state_dict(sd, device)
    else:
        block = net.packed().to(device)
        mode = _lib.PM_FOLD_TRAIN if net.training else _lib.PM_FOLD_EVAL
    return fold(block, mode)[0]


def run_episodes(env_kw, w_opp, opp_id, w_B, serves, device="cuda", max_steps=1_000_000):
    """One greedy episode per arena, each played start to finish inside the match megakernel
    (K8, pongmi.play). serves [E, 3] (vx, vy, spin) per episode; w_opp [nets, NW] with opp_id [E]
    (None: net 0) for player A, w_B for player B. Returns (wins [E] bool: rB > rA on the episode's
    last step, lengths [E] int) as host numpy arrays."""
    from .play import play
    E = int(np.asarray(serves).reshape(-1, 3).shape[0])
    n_opp = int(w_opp.shape[0])
    w_nets = torch.cat([w_opp.reshape(n_opp, -1), w_B.reshape(1, -1)]).to(device)
    netA = np.zeros(E, np.int64) if opp_id is None else np.asarray(torch.as_tensor(opp_id).cpu(), np.int64)
    _, _, length, last = play(env_kw, w_nets, netA, np.full(E, n_opp), serves, device, max_steps)
    return last > 0, length


def run_episodes_stepped(env_kw, w_opp, opp_id, w_B, serves, device="cuda", max_steps=1_000_000, check_every=16):
    """run_episodes as one act launch (K2) + one env launch (K1) per tick, all arenas in lockstep."""
    E = int(serves.shape[0])
    env = PongEnv2PBatch(E, device=device, serve_table=np.asarray(serves, np.float64).reshape(E, 1, 3),
                         autoreset=False, **env_kw)
    obsA, obsB = env.reset()
    finished = torch.zeros(E, dtype=torch.bool, device=device)
    wins = torch.zeros(E, dtype=torch.bool, device=device)
    length = torch.zeros(E, dtype=torch.int32, device=device)
    if opp_id is not None:
        opp_id = torch.as_tensor(opp_id, dtype=torch.int32).to(device)
    for t in range(max_steps):
        aA, aB = qnet_act(w_opp, opp_id, w_B, obsA, obsB, epsilon=-1.0)  # both greedy (argmax, first max)
        (obsA, obsB), (rA, rB), done, _ = env.step(aA, aB)
        new = done.bool() & ~finished
        wins |= new & (rB > rA)
        length = torch.where(new, torch.full_like(length, t + 1), length)
        finished |= new
        if (t + 1) % check_every == 0 and bool(finished.all()):
            break
    if not bool(finished.all()):
        raise RuntimeError(f"evaluation did not finish within {max_steps} steps")
    return wins.cpu().numpy(), length.cpu().numpy()


def eval_vs_model(env, A, B, episodes, *, rng=None, device="cuda", return_details=False):
    """Win rate of B against A over `episodes` greedy episodes (train_iterative.py:171-181)."""
    rng = _pyrandom if rng is None else rng
    kw = env_kwargs(env)
    cfg = env_config(**kw)
    serves = np.array([draw_serve(rng, cfg) for _ in range(int(episodes))], np.float64).reshape(-1, 3)
    w_A = folded_weights(A, device).reshape(1, -1)
    w_B = folded_weights(B, device)
    wins, length = run_episodes(kw, w_A, None, w_B, serves, device)
    rate = float(wins.sum()) / int(episodes)
    return (rate, wins, length) if return_details else rate


def eval_vs_pool(env, B, pool, episodes, *, rng=None, device="cuda", return_details=False):
    """Win rate of B against opponents drawn per episode from `pool` (train_iterative.py:183-196);
    1.0 for an empty pool, as the reference returns."""
    if not pool:
        return 1.0
    rng = _pyrandom if rng is None else rng
    kw = env_kwargs(env)
    cfg = env_config(**kw)
    opp = np.zeros(int(episodes), np.int32)
    serves = np.zeros((int(episodes), 3), np.float64)
    for e in range(int(episodes)):
        opp[e] = rng.choice(range(len(pool)))  # random.choice(pool): the same _randbelow draw
        serves[e] = draw_serve(rng, cfg)
    w_opp = torch.stack([folded_weights(p, device) for p in pool])
    w_B = folded_weights(B, device)
    wins, length = run_episodes(kw, w_opp, opp, w_B, serves, device)
    rate = float(wins.sum()) / int(episodes)
    return (rate, wins, length, opp) if return_details else rate
