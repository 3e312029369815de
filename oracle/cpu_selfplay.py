"""ORACLE — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

A plain CPU port of the batched self-play vector step (the same workload bench.py measures on the
GPU): both players act (numpy float32 MLPs, epsilon-greedy), every arena ticks (the C oracle of
envs/my_pong_env_2p.py), transitions go to a numpy PER ring (scripts/train_iterative.py:49-76),
then one double-DQN update of `batch` (train_iterative.py:132-168, numpy) with Adam. Used only
as bench.py's `cpu_baseline` ("kind": "port"), on one core.
"""
import numpy as np

from . import oracle as orc


def _eff32(sd, noisy, eps=None):
    e = orc.qnet_effective(sd, noisy, eps)
    return {k: np.asarray(v, np.float32) for k, v in e.items()}


def _q32(e, x):
    h = np.maximum(x @ e["W1"].T + e["b1"], 0)
    h = np.maximum(h @ e["W2"].T + e["b2"], 0)
    V = h @ e["fc_V.W"].T + e["fc_V.b"]
    A = h @ e["fc_A.W"].T + e["fc_A.b"]
    return V + (A - A.mean(1, keepdims=True))


class CpuSelfPlay:
    def __init__(self, env_kw, n, sdB, sdA, pool_sds, batch=256, cap=1_000_000, epsilon=0.02, pool_ratio=0.33,
                 seed=0, gamma=0.99, lr=2.5e-4):
        self.rng = np.random.RandomState(seed)
        self.pv = orc.env_params_from_kwargs(**env_kw)
        self.P = orc.make_params(self.pv)
        self.n, self.batch, self.cap = n, batch, cap
        self.sdB = {k: np.asarray(v, np.float32) for k, v in sdB.items()}
        self.effA = _eff32({k: np.asarray(v) for k, v in sdA.items()}, True)
        self.effP = [_eff32({k: np.asarray(v) for k, v in s.items()}, False) for s in pool_sds]
        self.heads = orc.pack_heads(self.sdB)
        self.target = self.heads.copy()
        self.m = np.zeros_like(self.heads)
        self.v = np.zeros_like(self.heads)
        self.t = 0
        self.eps, self.pool_ratio, self.gamma, self.lr = epsilon, pool_ratio, gamma, lr
        self.arr = np.zeros(n, orc.ARENA_DTYPE)
        self.opp = np.zeros(n, np.int64)
        self._serve(np.ones(n, bool))
        self.s = np.zeros((cap, 7), np.float32)
        self.ns = np.zeros((cap, 7), np.float32)
        self.a = np.zeros(cap, np.int64)
        self.r = np.zeros(cap, np.float32)
        self.d = np.zeros(cap, bool)
        self.prios = np.zeros(cap, np.float32)
        self.pos = self.size = 0
        self.frame = 0

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
        use = (self.rng.rand(k) < self.pool_ratio) & (len(self.effP) > 0)
        self.opp[mask] = np.where(use, 1 + self.rng.randint(0, max(len(self.effP), 1), k), 0)

    def step(self):
        n = self.n
        oA, oB = orc.obs_of_arenas(self.arr)
        qa = np.empty((n, 3), np.float32)
        for k, e in enumerate([self.effA] + self.effP):
            sel = self.opp == k
            if sel.any():
                qa[sel] = _q32(e, oA[sel])
        wn = orc.noise_from_raw(self.rng.randn(64).astype(np.float32), self.rng.randn(1).astype(np.float32))
        an = orc.noise_from_raw(self.rng.randn(64).astype(np.float32), self.rng.randn(3).astype(np.float32))
        eps_act = {"fc_V.weight_epsilon": wn[0], "fc_V.bias_epsilon": wn[1], "fc_A.weight_epsilon": an[0],
                   "fc_A.bias_epsilon": an[1]}
        qb = _q32(_eff32({**self.sdB, **orc.unpack_heads(self.heads.astype(np.float32))}, True, eps_act), oB)
        aA = np.argmax(qa, 1).astype(np.int8)
        aB = np.where(self.rng.rand(n) < self.eps, self.rng.randint(0, 3, n), np.argmax(qb, 1)).astype(np.int8)
        nA, nB, rew, done = orc.step_arenas(self.P, self.arr, aA, aB)
        slots = (self.pos + np.arange(n)) % self.cap
        self.s[slots], self.ns[slots], self.a[slots], self.r[slots], self.d[slots] = oB, nB, aB, rew[:, 1], done > 0
        self.prios[slots] = self.prios.max() if self.size else 1.0
        self.pos = (self.pos + n) % self.cap
        self.size = min(self.size + n, self.cap)
        self._serve(done > 0)
        D = int(done.sum())
        self.eps = max(0.02, self.eps * 0.995 ** D)
        if self.size >= self.batch:
            self.frame += 1
            beta = min(1.0, 0.4 + self.frame * 0.6 / 100000)
            idx, w = orc.per_sample(self.prios, self.size, self.batch, beta, self.rng.random_sample(self.batch))
            tn = orc.noise_from_raw(self.rng.randn(64).astype(np.float32), self.rng.randn(1).astype(np.float32))
            ta = orc.noise_from_raw(self.rng.randn(64).astype(np.float32), self.rng.randn(3).astype(np.float32))
            eps_tr = {"fc_V.weight_epsilon": tn[0], "fc_V.bias_epsilon": tn[1], "fc_A.weight_epsilon": ta[0],
                      "fc_A.bias_epsilon": ta[1]}
            res = orc.dqn_loss_grads(self.sdB, self.heads, self.target, eps_tr, self.s[idx], self.a[idx], self.r[idx],
                                     self.ns[idx], self.d[idx], w, self.gamma)
            self.t += 1
            self.heads, self.m, self.v = orc.adam_step(self.heads, res["grads"], self.m, self.v, self.t, self.lr)
            orc.per_update(self.prios, idx, res["errors"])
            if self.t % 1000 == 0:
                self.target = self.heads.copy()
        return n


class CpuRollout:
    """BASELINE configs[1] on the CPU: the inference-only rollout (scripts/train_iterative.py:239-242
    with the learner off) for n arenas — modelA greedy on folded weights, modelB epsilon-greedy with
    fresh NoisyNet noise per vector step (select_action_B, :125-130), the C oracle's tick, reset on
    done. bench.py --workload infer's `cpu_baseline` ("kind": "port"), on one core."""

    def __init__(self, env_kw, n, sdB, sdA, epsilon=0.02, seed=0, replay_cap=0):
        self.rng = np.random.RandomState(seed)
        # replay_cap > 0: bench --workload collect's baseline — every transition is also pushed, as
        # memory.push((oB, aB, rB, nB, done)) (:242-243, :56-63), into a [cap][16] f32 ring with its
        # priority (max priority, 1.0 here: no learner) and PER leaf prio ** 0.6
        self.cap = int(replay_cap)
        if self.cap:
            self.trans = np.zeros((self.cap, 16), np.float32)
            self.prios = np.zeros(self.cap, np.float32)
            self.leaves = np.zeros(self.cap, np.float32)
            self.ep_reward = np.zeros(n, np.float32)
            self.pos = 0
        self.pv = orc.env_params_from_kwargs(**env_kw)
        self.P = orc.make_params(self.pv)
        self.n, self.eps = n, epsilon
        self.sdB = {k: np.asarray(v, np.float32) for k, v in sdB.items()}
        self.effA = _eff32({k: np.asarray(v) for k, v in sdA.items()}, True)
        self.arr = np.zeros(n, orc.ARENA_DTYPE)
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

    def step(self):
        n = self.n
        oA, oB = orc.obs_of_arenas(self.arr)
        wn = orc.noise_from_raw(self.rng.randn(64).astype(np.float32), self.rng.randn(1).astype(np.float32))
        an = orc.noise_from_raw(self.rng.randn(64).astype(np.float32), self.rng.randn(3).astype(np.float32))
        eps_act = {"fc_V.weight_epsilon": wn[0], "fc_V.bias_epsilon": wn[1], "fc_A.weight_epsilon": an[0],
                   "fc_A.bias_epsilon": an[1]}
        qb = _q32(_eff32(self.sdB, True, eps_act), oB)
        aA = np.argmax(_q32(self.effA, oA), 1).astype(np.int8)
        aB = np.where(self.rng.rand(n) < self.eps, self.rng.randint(0, 3, n), np.argmax(qb, 1)).astype(np.int8)
        _, nB, rew, done = orc.step_arenas(self.P, self.arr, aA, aB)
        if self.cap:
            slot = (self.pos + np.arange(n)) % self.cap
            row = self.trans[slot]
            row[:, 0:7] = oB
            row[:, 7] = rew[:, 1]
            row[:, 8:15] = nB
            row[:, 15] = (aB.astype(np.int32) | (done.astype(np.int32) << 8)).view(np.float32)
            self.trans[slot] = row
            self.prios[slot] = 1.0
            self.leaves[slot] = np.float32(1.0) ** np.float32(0.6)
            self.pos = (self.pos + n) % self.cap
            self.ep_reward += rew[:, 1]
            self.ep_reward[done > 0] = 0.0
        self._serve(done > 0)
        return n


class PhiloxRollout:
    """TEST ORACLE for K9 (pm_rollout) and the collecting rollout (pm_rollout_push): the
    rollout of scripts/train_iterative.py:239-245 with the learner off, restated on the device's own
    random streams and float32 order so a launch can be compared with it bit for bit, independently of
    every other device path. Per vector step with counter c:
      - modelB.reset_noise() (select_action_B, :125): the Philox noise of (seed_net, TAG_NOISE_ACT, c)
        (oracle.philox_noise, bit-exact with the device's normal()), folded mu + sigma * eps in torch's
        float32 order (fold_heads_f32);
      - both forwards in the matrix-core tile's fmaf order (qnet_forward_f32); modelA greedy on its own
        frozen epsilon buffers (:240), modelB eps-greedy with the Philox draw of (arena, TAG_ACT, c)
        (:126-130);
      - env.step on the C oracle (envs/my_pong_env_2p.py:116-225), finished arenas served again from
        the step-keyed Philox serve (oracle.philox_serve(step=c));
      - with a replay ring: memory.push((oB, aB, rB, nB, done)) (:242-243, PrioritizedReplay.push
        :56-63) into slot (pos + s n + i) % cap with the given push priority; ep_reward += rB, and the
        episode wins ep_reward > 0 (:245-249).
    The start state is the device env's (get_state()), so the launch's input is shared and nothing
    else is."""

    def __init__(self, env_kw, state, sdA, sdB, epsilon, seed_env, seed_net, counter, replay=None):
        self.pv = orc.env_params_from_kwargs(**env_kw)
        self.P = orc.make_params(self.pv)
        self.arr = np.zeros(len(state["x"]), orc.ARENA_DTYPE)
        for k in ("x", "y", "vx", "vy", "spin", "top", "bot", "scoreA", "scoreB", "bounces"):
            self.arr[k] = state[k]
        self.n = len(self.arr)
        f = lambda sd: {k: np.asarray(v, np.float32) for k, v in sd.items()}  # noqa: E731
        self.sdB = f(sdB)
        self.wA = orc.fold_heads_f32(f(sdA), "train")
        self.eps, self.seed_env, self.seed_net, self.counter = float(epsilon), int(seed_env), int(seed_net), int(counter)
        self.replay = replay  # dict(trans [cap,16] f32, prios [cap] f32, pos, cap, prio) or None
        self.ep_reward = np.zeros(self.n, np.float32)
        self.stats = np.zeros(6, np.int64)  # episodes, done & rB > 0, points A, points B, episode wins, reward sum

    def heads_B(self, c):
        fVi, fVo, fAi, fAo = orc.philox_noise(self.seed_net, orc.TAG_NOISE_ACT, c)
        eps = {"fc_V.weight_epsilon": np.outer(fVo, fVi).astype(np.float32), "fc_V.bias_epsilon": fVo,
               "fc_A.weight_epsilon": np.outer(fAo, fAi).astype(np.float32), "fc_A.bias_epsilon": fAo}
        return orc.fold_heads_f32({**self.sdB, **eps}, "train")

    def step(self, s=0):
        n, c = self.n, self.counter
        arenas = np.arange(n)
        oA, oB = orc.obs_of_arenas(self.arr)
        aA = orc.argmax_first(orc.qnet_forward_f32(self.wA, oA))
        aB, _ = orc.eps_greedy(orc.qnet_forward_f32(self.heads_B(c), oB), self.eps, self.seed_env, c, arenas)
        _, nB, rew, done = orc.step_arenas(self.P, self.arr, aA.astype(np.int8), aB.astype(np.int8))
        d = done.astype(bool)
        rA, rB = rew[:, 0], rew[:, 1]
        if self.replay is not None:
            R = self.replay
            slot = (R["pos"] + s * n + arenas) % R["cap"]
            R["trans"][slot, 0:7] = oB
            R["trans"][slot, 7] = rB
            R["trans"][slot, 8:15] = nB
            R["trans"][slot, 15] = (aB.astype(np.int32) | (d.astype(np.int32) << 8)).view(np.float32)
            R["prios"][slot] = R["prio"]
        self.ep_reward += rB
        self.stats += np.array([d.sum(), (d & (rB > 0)).sum(), (rA > 0).sum(), (rB > 0).sum(),
                                (d & (self.ep_reward > 0)).sum(), int(self.ep_reward[d].sum())])
        self.ep_reward[d] = 0.0
        if d.any():
            i = np.nonzero(d)[0]
            vx, vy, spin = orc.philox_serve(self.pv, i, None, self.seed_env, step=c)
            orc.serve_arenas(self.arr, d, vx, vy, spin)
        self.counter += 1
        return aA, aB

    def run(self, steps):
        for s in range(steps):
            self.step(s)
        if self.replay is not None:
            self.replay["pos"] = (self.replay["pos"] + steps * self.n) % self.replay["cap"]
        return self.stats
