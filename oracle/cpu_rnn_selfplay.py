"""ORACLE — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

A plain CPU port of the batched QNetRNN self-play vector step (scripts/train_rnn_iterative.py:731-798,
the workload `bench.py --workload rnn` measures on the GPU): both players act with QNetRNN (numpy
float32, (h, c) carried per arena, zeroed at episode start; B epsilon-greedy with fresh NoisyLinear
noise per step), every arena ticks (the C oracle of envs/my_pong_env_2p.py), transitions go to
per-arena rings and finished episodes of length >= T to a deque (SequenceReplayBuffer, :100-176),
then one DRQN update of 64 x 8 (oracle.drqn_update, float64 numpy) once the buffer holds enough
episodes. Used only as bench.py's `cpu_baseline` ("kind": "port"), on one core.
"""
from collections import deque

import numpy as np

from . import oracle as orc


def _eff32(sd, train, noise=None):
    sd = dict(sd)
    if noise is not None:
        sd.update(noise)
    return {k: np.asarray(v, np.float32) for k, v in orc.rnn_effective(sd, train).items()}


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def _step32(e, x, h, c):
    f1 = np.maximum(x @ e["W1"].T + e["b1"], 0)
    f2 = np.maximum(f1 @ e["W2"].T + e["b2"], 0)
    z = f2 @ e["Wih"].T + e["bih"] + h @ e["Whh"].T + e["bhh"]
    i, f, g, o = np.split(z, 4, axis=1)
    c2 = _sig(f) * c + _sig(i) * np.tanh(g)
    h2 = _sig(o) * np.tanh(c2)
    s = np.maximum(h2 @ e["S.W"].T + e["S.b"], 0)
    V = s @ e["V.W"].T + e["V.b"]
    A = s @ e["A.W"].T + e["A.b"]
    return V + (A - A.mean(1, keepdims=True)), h2, c2


def _noise(rng):
    f = lambda x: np.sign(x) * np.sqrt(np.abs(x))  # noqa: E731  _scale_noise (models/qnet_rnn.py:33-35)
    out = {}
    for key, n_in, n_out in (("fc_shared_head.0", 128, 128), ("fc_V", 128, 1), ("fc_A", 128, 3)):
        e_in = f(rng.randn(n_in).astype(np.float32))
        e_out = f(rng.randn(n_out).astype(np.float32))
        out[f"{key}.weight_epsilon"] = np.outer(e_out, e_in)
        out[f"{key}.bias_epsilon"] = e_out
    return out


class CpuRnnSelfPlay:
    def __init__(self, env_kw, n, sdB, sdA, pool_sds, batch=64, T=8, cap=200_000, min_episodes=640, depth=1024,
                 epsilon=0.05, pool_ratio=0.4, seed=0, gamma=0.99, lr=1e-4):
        self.rng = np.random.RandomState(seed)
        self.pv = orc.env_params_from_kwargs(**env_kw)
        self.P = orc.make_params(self.pv)
        self.n, self.batch, self.T, self.depth, self.min_episodes = n, batch, T, depth, min_episodes
        self.sdB = {k: np.asarray(v, np.float64) for k, v in sdB.items()}
        self.target = dict(self.sdB)
        self.effO = [_eff32(sdA, False)] + [_eff32(s, False) for s in pool_sds]
        self.adam, self.t = {}, 0
        self.eps, self.pool_ratio, self.gamma, self.lr = epsilon, pool_ratio, gamma, lr
        self.arr = np.zeros(n, orc.ARENA_DTYPE)
        self.opp = np.zeros(n, np.int64)
        self.hA, self.cA, self.hB, self.cB = (np.zeros((n, 128), np.float32) for _ in range(4))
        self.ep_len = np.zeros(n, np.int64)
        self.ring = np.zeros((depth, n, 16), np.float32)
        self.episodes = deque(maxlen=cap)
        self.step_idx = 0
        self._serve(np.ones(n, bool))

    def _serve(self, mask):
        k = int(mask.sum())
        if k == 0:
            return
        p = self.pv
        speed = self.rng.uniform(p["speed_lo"], p["speed_hi"], k)
        coin = self.rng.rand(k) < 0.5
        ang = np.where(coin, self.rng.uniform(p["ang0_lo"], p["ang0_hi"], k), self.rng.uniform(p["ang1_lo"], p["ang1_hi"], k))
        rad = np.radians(ang)
        orc.serve_arenas(self.arr, mask, speed * np.cos(rad), speed * np.sin(rad),
                         self.rng.uniform(p["spin_lo"], p["spin_hi"], k))
        use = (self.rng.rand(k) < self.pool_ratio) & (len(self.effO) > 1)
        self.opp[mask] = np.where(use, 1 + self.rng.randint(0, max(len(self.effO) - 1, 1), k), 0)
        for s in (self.hA, self.cA, self.hB, self.cB):
            s[mask] = 0

    def step(self):
        n = self.n
        oA, oB = orc.obs_of_arenas(self.arr)
        qa = np.empty((n, 3), np.float32)
        for k, e in enumerate(self.effO):
            sel = self.opp == k
            if sel.any():
                qa[sel], self.hA[sel], self.cA[sel] = _step32(e, oA[sel], self.hA[sel], self.cA[sel])
        effB = _eff32(self.sdB, True, _noise(self.rng))
        qb, self.hB, self.cB = _step32(effB, oB, self.hB, self.cB)
        aA = np.argmax(qa, 1).astype(np.int8)
        aB = np.where(self.rng.rand(n) < self.eps, self.rng.randint(0, 3, n), np.argmax(qb, 1)).astype(np.int8)
        nA, nB, rew, done = orc.step_arenas(self.P, self.arr, aA, aB)
        slot = self.step_idx % self.depth
        self.ring[slot, :, 0:7], self.ring[slot, :, 7], self.ring[slot, :, 8:15] = oB, rew[:, 1], nB
        self.ring[slot, :, 15] = aB.astype(np.int64) + 256 * done.astype(np.int64)
        self.ep_len += 1
        d = done > 0
        for i in np.nonzero(d & (self.ep_len >= self.T))[0]:
            self.episodes.append((i, self.step_idx - self.ep_len[i] + 1, self.ep_len[i]))
        for _ in range(int(d.sum())):
            self.eps = max(0.05, self.eps * 0.999)
        self.ep_len[d] = 0
        self._serve(d)
        self.step_idx += 1
        if len(self.episodes) > self.min_episodes:
            self._update()
        return n

    def _update(self):
        B, T = self.batch, self.T
        pick = self.rng.choice(len(self.episodes), B, replace=True)
        rows = np.empty((B, T, 16), np.float32)
        for b, j in enumerate(pick):
            arena, start, length = self.episodes[j]
            st = start + self.rng.randint(0, length - T + 1)
            rows[b] = self.ring[(st + np.arange(T)) % self.depth, arena]
        bits = rows[..., 15].astype(np.int64)
        batch = (rows[..., 0:7], bits % 256, rows[..., 7], rows[..., 8:15], bits >= 256)
        self.t += 1
        self.sdB, _ = orc.drqn_update(self.sdB, self.target, self.adam, self.t, batch, lr=self.lr, gamma=self.gamma)
        if self.t % 2000 == 0:
            self.target = dict(self.sdB)
