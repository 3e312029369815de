"""Batched round-robin tournament: tests/test_round_robin.py (:117-386) with every (pair, episode)
as one arena of a PongEnv2PBatch advanced in lockstep.

The reference plays the pairs (i < j, participant order) one episode after another on one
PongEnv2P: each episode is env.reset() (its serve drawn from the global `random` stream) and greedy
play until done; the winner is decided by the final scoreA / scoreB (:317-321). Here the host draws
every episode's serve from the same stream in the same order, so episode e of pair p sees exactly
the serve the reference's would, and all episodes run at once:

  * episodes between QNet / ball-follower players run start to finish in the match megakernel
    (K8, pongmi.play: both nets staged per block, arenas in registers, one launch);
  * in episodes with a QNetRNN player, QNet participants act through pm_qnet_q on their arenas
    (eval mode: NoisyLinear mu, as load_model_universal leaves them, :181-185);
  * QNetRNN participants through pm_rnn_q with (h, c) per arena and side, from zero state;
  * HardcodedBallFollower through the same comparison as :207-228 (float32, numpy 2 semantics).

load_model_universal keeps the reference's checkpoint key order, its legacy fc.* -> dueling mapping
(:144-168) and strictness, and loads with torch.load(weights_only=True). The returned frames have
the reference's columns and order (match records: pair-major, episode 1..E; summary: by win_rate).
"""
import itertools
import random as _pyrandom
from pathlib import Path

import numpy as np
import torch

from . import _lib
from . import qnet as _qnet
from . import rnn as _rnn
from .env import PongEnv2PBatch, draw_serve, env_config

STATE_KEYS = ["modelB_state", "modelA_state", "modelB", "modelA", "model", "state_dict"]
HARDCODED = "HardcodedBallFollower"


def _state_dict_of(ckpt, name, path):
    for key in STATE_KEYS:
        if key in ckpt:
            return ckpt[key]
    if all(not isinstance(v, dict) for v in ckpt.values()) and any(
            k.startswith("fc.") or k.startswith("features.") for k in ckpt.keys()):
        return ckpt
    raise KeyError(f"no model state dict in checkpoint of '{name}' ({path}); tried {STATE_KEYS}, "
                   f"keys {list(ckpt.keys())}")


def load_model_universal(model_info, rnn_arch_config, device):
    """A QNet / QNetRNN drop-in module in eval mode (test_round_robin.py:117-185), or the string
    "HardcodedAgent" for the ball follower."""
    from models.qnet import QNet
    from models.qnet_rnn import QNetRNN
    typ = model_info["type"]
    name = model_info.get("name", Path(model_info["path"]).stem)
    if typ == HARDCODED:
        return "HardcodedAgent"
    path = Path(model_info["path"])
    if not path.exists():
        raise FileNotFoundError(f"model '{name}' not found at {path}")
    sd = _state_dict_of(torch.load(path, map_location="cpu", weights_only=True), name, path)
    if typ == "QNet":
        net = QNet(input_dim=7, output_dim=3)
        if any(k.startswith(("features.", "fc_V.", "fc_A.")) for k in sd):
            net.load_state_dict(sd, strict=True)
        else:  # legacy fc.0 / fc.2 / fc.4 checkpoints: features copied, fc.4 becomes the advantage mu
            mapped = {}
            for k, v in sd.items():
                if k.startswith("fc.0."):
                    mapped[k.replace("fc.0.", "features.0.")] = v
                elif k.startswith("fc.2."):
                    mapped[k.replace("fc.2.", "features.2.")] = v
            if "fc.4.weight" in sd and "fc.4.bias" in sd:
                w4, b4 = sd["fc.4.weight"], sd["fc.4.bias"]
                mapped["fc_A.weight_mu"], mapped["fc_A.bias_mu"] = w4, b4
                mapped["fc_V.weight_mu"], mapped["fc_V.bias_mu"] = w4.mean(dim=0, keepdim=True), b4.mean().unsqueeze(0)
            net.load_state_dict(mapped, strict=False)
    elif typ == "QNetRNN":
        cfg = rnn_arch_config or {}
        net = QNetRNN(input_dim=7, output_dim=3, feature_dim=cfg.get("feature_dim", 128),
                      lstm_hidden_dim=cfg.get("lstm_hidden_dim", 128), lstm_layers=cfg.get("lstm_layers", 1),
                      head_hidden_dim=cfg.get("head_hidden_dim", 128))
        net.load_state_dict(sd)
    else:
        raise ValueError(f"unsupported model type '{typ}' (model {name})")
    net.eval()
    net.reset_noise()
    return net.to(device)


class _Player:
    """One participant's acting on the arenas where it plays side A and side B."""

    def __init__(self, model, typ, rows_A, rows_B, device):
        self.typ = typ
        self.rows = (rows_A, rows_B)
        if typ == "QNet":
            self.w = _qnet.fold(model.packed().to(device), _lib.PM_FOLD_EVAL)[0]
        elif typ == "QNetRNN":
            self.w = _rnn.fold(model.packed().to(device), _lib.PM_FOLD_EVAL)[0]
            self.state = [_rnn.init_state(int(r.numel()), device) for r in self.rows]

    def act(self, side, obs, out):
        rows = self.rows[side]
        if rows.numel() == 0:
            return
        x = obs.index_select(0, rows)
        if self.typ == "QNet":
            a = _qnet.q_values(self.w, x).argmax(1)
        elif self.typ == "QNetRNN":
            h, c = self.state[side]
            a = _rnn.q_step(self.w, x, h, c).argmax(1)
        else:  # ball follower: obs = (ball_x, ball_y, vx, vy, my_paddle_x, other_paddle_x, spin)
            ball, mine = x[:, 0], x[:, 4]
            tol = torch.tensor(0.01, dtype=torch.float32, device=x.device)
            a = torch.where(ball < mine - tol, 0, torch.where(ball > mine + tol, 2, 1))
        out.index_copy_(0, rows, a.to(out.dtype))


def play_matches(env_params, models, plan, device="cuda", rng=None, max_steps=1_000_000):
    """Play every episode of `plan` at once. models: name -> (module or "HardcodedAgent", type);
    plan: [(name_A, name_B, episodes)] in the order the reference plays them (its serves are drawn
    from `rng` / the global random stream in that order, one env.reset() per episode).
    Episodes between QNet / ball-follower players run in the match megakernel (K8, pongmi.play);
    episodes with a QNetRNN player step all their arenas in lockstep (K5 + K1 per tick).
    Returns [(name_A, name_B, score_A, score_B)] per episode, in plan order."""
    rng = _pyrandom if rng is None else rng
    env_kw = {k: v for k, v in dict(env_params).items() if k not in ("render_size", "enable_render")}
    cfg = env_config(**env_kw)
    eps = [(a, b) for a, b, e in plan for _ in range(int(e))]
    n = len(eps)
    if n == 0:
        return []
    serves = np.array([draw_serve(rng, cfg) for _ in range(n)], np.float64).reshape(n, 3)
    score = np.zeros((n, 2), np.int64)
    rnn = {nm for nm, (_, typ) in models.items() if typ == "QNetRNN"}
    stepped = np.array([a in rnn or b in rnn for a, b in eps], bool)
    if (~stepped).any():
        score[~stepped] = _play_fused(env_kw, models, [eps[k] for k in np.nonzero(~stepped)[0]], serves[~stepped],
                                      device, max_steps)
    if stepped.any():
        score[stepped] = _play_stepped(env_kw, models, [eps[k] for k in np.nonzero(stepped)[0]], serves[stepped],
                                       device, max_steps)
    return [(a, b, int(score[k, 0]), int(score[k, 1])) for k, (a, b) in enumerate(eps)]


def _play_fused(env_kw, models, eps, serves, device, max_steps):
    """QNet / ball-follower episodes in the match megakernel: [E, 2] final scores."""
    from .play import FOLLOWER, play
    ids, weights = {}, []
    for nm in dict.fromkeys([x for ab in eps for x in ab]):
        module, typ = models[nm]
        if typ == HARDCODED:
            ids[nm] = FOLLOWER
        else:  # eval mode: NoisyLinear mu (load_model_universal leaves the nets in eval, :181-185)
            ids[nm] = len(weights)
            weights.append(_qnet.fold(module.packed().to(device), _lib.PM_FOLD_EVAL)[0])
    w = torch.stack(weights) if weights else None
    sA, sB, _, _ = play(env_kw, w, [ids[a] for a, _ in eps], [ids[b] for _, b in eps], serves, device, max_steps)
    return np.stack([sA, sB], 1)


def _play_stepped(env_kw, models, eps, serves, device, max_steps):
    """Episodes with a QNetRNN player: all arenas in lockstep, one act per participant and side plus
    one env launch per tick: [E, 2] final scores."""
    n = len(eps)
    names = list(dict.fromkeys([x for ab in eps for x in ab]))
    index = {nm: k for k, nm in enumerate(names)}
    ida = torch.tensor([index[a] for a, _ in eps], dtype=torch.int64, device=device)
    idb = torch.tensor([index[b] for _, b in eps], dtype=torch.int64, device=device)
    players = [_Player(models[nm][0], models[nm][1], (ida == k).nonzero().flatten(), (idb == k).nonzero().flatten(),
                       device) for k, nm in enumerate(names)]
    env = PongEnv2PBatch(n, device=device, serve_table=serves.reshape(n, 1, 3), autoreset=False, **env_kw)
    obsA, obsB = env.reset()
    aA = torch.zeros(n, dtype=torch.int8, device=device)
    aB = torch.zeros(n, dtype=torch.int8, device=device)
    finished = torch.zeros(n, dtype=torch.bool, device=device)
    score = torch.zeros((n, 2), dtype=torch.int32, device=device)
    for t in range(max_steps):
        for pl in players:
            pl.act(0, obsA, aA)
            pl.act(1, obsB, aB)
        (obsA, obsB), _, done, _ = env.step(aA, aB)
        new = done.bool() & ~finished
        score = torch.where(new.unsqueeze(1), env.i32[0:2].t(), score)
        finished |= new
        if (t + 1) % 16 == 0 and bool(finished.all()):
            break
    if not bool(finished.all()):
        raise RuntimeError(f"matches did not finish within {max_steps} steps")
    return score.cpu().numpy()


def summarize(records, names, key="name"):
    """win / lose / draw / games_played / win_rate per participant, sorted by win_rate (:351-386)."""
    import pandas as pd
    stats = {nm: {"win": 0, "lose": 0, "draw": 0, "games_played": 0} for nm in names}
    for a, b, w in records:
        stats[a]["games_played"] += 1
        stats[b]["games_played"] += 1
        if w == a:
            stats[a]["win"] += 1
            stats[b]["lose"] += 1
        elif w == b:
            stats[b]["win"] += 1
            stats[a]["lose"] += 1
        else:
            stats[a]["draw"] += 1
            stats[b]["draw"] += 1
    rows = [{key: nm, **s, "win_rate": (s["win"] / s["games_played"]) if s["games_played"] else 0}
            for nm, s in stats.items()]
    return pd.DataFrame(rows).sort_values("win_rate", ascending=False).set_index(key)


def run_round_robin_tournament(env_params, rnn_arch_params, models_to_compete, episodes_per_match, device="cuda",
                               verbose_progress=False, rng=None, max_steps=1_000_000):
    """(match_df, summary_df) as test_round_robin.py:238-386 returns them."""
    import pandas as pd
    participants = {}
    for info in models_to_compete:
        try:
            participants[info["name"]] = (load_model_universal(info, rnn_arch_params, device), info["type"])
        except Exception as e:  # the reference skips models that fail to load (:259-261)
            print(f"  [error] loading '{info['name']}' failed: {e}")
    if len(participants) < 2:
        return pd.DataFrame(), pd.DataFrame(columns=["name", "win", "lose", "draw", "games_played", "win_rate"])
    names = list(participants)
    E = int(episodes_per_match)
    plan = [(a, b, E) for a, b in itertools.combinations(names, 2)]
    played = play_matches(env_params, participants, plan, device, rng, max_steps)
    records, k = [], 0
    for a, b, e in plan:
        for ep in range(e):
            _, _, sA, sB = played[k]
            k += 1
            winner = a if sA > sB else b if sB > sA else "draw"
            records.append({"episode": ep + 1, "player_A_name": a, "player_B_name": b,
                            "player_A_type": participants[a][1], "player_B_type": participants[b][1],
                            "score_A": sA, "score_B": sB, "winner_name": winner})
            if verbose_progress:
                print(f"  {a} vs {b} episode {ep + 1}: {sA}-{sB}, winner {winner}")
    match_df = pd.DataFrame(records)
    summary_df = summarize([(r["player_A_name"], r["player_B_name"], r["winner_name"]) for r in records], names)
    return match_df, summary_df


def save_results(match_df, summary_df, output_dir, timestamp):
    """match_records_<ts>.csv and summary_ranking_<ts>.csv as the reference writes them (:497-501)."""
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    match_path = out / f"match_records_{timestamp}.csv"
    summary_path = out / f"summary_ranking_{timestamp}.csv"
    match_df.to_csv(match_path, index=False)
    summary_df.to_csv(summary_path)
    return match_path, summary_path
