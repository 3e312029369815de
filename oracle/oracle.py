"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's hot path, used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the CHECKER (never as the thing measured on the GPU, never
imported by the product package `pingpong-selfplay-ai_amd/`).

  env / physics / CPython `random`  -> C (oracle/pong_oracle.c, built into oracle/_build/liborcpong.so)
  QNet forward                      -> numpy, float64        models/qnet.py:43-50,71-75
  QNetRNN forward (LSTM)            -> numpy, float64        models/qnet_rnn.py:43-50,107-144
  NoisyLinear.reset_noise transform -> numpy                 models/qnet.py:33-41
  PrioritizedReplay                 -> numpy                 scripts/train_iterative.py:49-76
  double-DQN train_step + Adam      -> numpy, float64        scripts/train_iterative.py:132-168,
                                                             torch.optim.Adam (torch 2.x single-tensor)

Pinned against tests/golden/*.npz produced from the reference by tests/golden/make_golden.py.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(HERE, "_build", "liborcpong.so")
_lib = None

ENV_PARAM_NAMES = ["paddle_width", "paddle_speed", "magnus_factor", "restitution", "friction", "ball_mass",
                   "world_ball_radius", "speed_lo", "speed_hi", "spin_lo", "spin_hi", "ang0_lo", "ang0_hi",
                   "ang1_lo", "ang1_hi", "speed_increment", "max_score", "speed_scale_every", "enable_spin"]


class OrParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in ENV_PARAM_NAMES[:16]] + \
               [("max_score", ctypes.c_int32), ("speed_scale_every", ctypes.c_int32),
                ("enable_spin", ctypes.c_int32), ("_pad", ctypes.c_int32)]


class OrArena(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in ("x", "y", "vx", "vy", "spin", "top", "bot")] + \
               [("scoreA", ctypes.c_int32), ("scoreB", ctypes.c_int32), ("bounces", ctypes.c_int32),
                ("_pad", ctypes.c_int32)]


class OrMT(ctypes.Structure):
    _fields_ = [("mt", ctypes.c_uint32 * 624), ("mti", ctypes.c_int)]


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(HERE, "pong_oracle.c")
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(_LIB_PATH)
        P, D, I32, U64 = ctypes.c_void_p, ctypes.c_double, ctypes.c_int32, ctypes.c_uint64
        L.or_collide.argtypes = [D] * 8 + [P]
        L.or_mt_seed.argtypes = [P, U64]
        L.or_mt_random.argtypes = [P]
        L.or_mt_random.restype = D
        L.or_mt_u32.argtypes = [P]
        L.or_mt_u32.restype = ctypes.c_uint32
        L.or_mt_randbelow.argtypes = [P, I32]
        L.or_mt_randbelow.restype = I32
        L.or_reset_draws.argtypes = [P, P, P]
        L.or_reset_apply.argtypes = [P, D, D, D]
        L.or_obs.argtypes = [P, P, P]
        L.or_step.argtypes = [P, P, I32, I32, P]
        L.or_step.restype = I32
        L.or_step_batch.argtypes = [P, P, P, P, P, P, P, P, I32]
        L.or_rollout_random.argtypes = [P, U64, ctypes.c_int64, P]
        L.or_rollout_random.restype = ctypes.c_int64
        L.or_qnet_f32.argtypes = [P, P, I32, P, P]
        L.or_argmax3.argtypes = [P, I32, P]
        for f in ("or_mt_sizeof", "or_params_sizeof", "or_arena_sizeof"):
            getattr(L, f).restype = I32
        assert L.or_mt_sizeof() == ctypes.sizeof(OrMT)
        assert L.or_params_sizeof() == ctypes.sizeof(OrParams)
        assert L.or_arena_sizeof() == ctypes.sizeof(OrArena)
        _lib = L
    return _lib


# ----------------------------------------------------------------------------- env params
def env_params_from_kwargs(**kw):
    """Same defaults as PongEnv2P.__init__ (envs/my_pong_env_2p.py:19-37)."""
    d = dict(paddle_width=0.2, paddle_speed=0.02, max_score=3, enable_spin=True, magnus_factor=0.01,
             restitution=0.9, friction=0.2, ball_mass=1.0, world_ball_radius=0.03, ball_speed_range=(0.01, 0.05),
             spin_range=(-10, 10), ball_angle_intervals=None, speed_scale_every=3, speed_increment=0.2)
    d.update({k: v for k, v in kw.items() if k in d})
    ai = d["ball_angle_intervals"] or [[-60, -30], [30, 60]]
    return dict(paddle_width=d["paddle_width"], paddle_speed=d["paddle_speed"], magnus_factor=d["magnus_factor"],
                restitution=float(d["restitution"]), friction=d["friction"], ball_mass=d["ball_mass"],
                world_ball_radius=d["world_ball_radius"], speed_lo=d["ball_speed_range"][0],
                speed_hi=d["ball_speed_range"][1], spin_lo=d["spin_range"][0], spin_hi=d["spin_range"][1],
                ang0_lo=ai[0][0], ang0_hi=ai[0][1], ang1_lo=ai[1][0], ang1_hi=ai[1][1],
                speed_increment=d["speed_increment"], max_score=int(d["max_score"]),
                speed_scale_every=int(d["speed_scale_every"]), enable_spin=int(bool(d["enable_spin"])))


def make_params(p):
    s = OrParams()
    for n in ENV_PARAM_NAMES:
        setattr(s, n, int(p[n]) if n in ("max_score", "speed_scale_every", "enable_spin") else float(p[n]))
    return s


# ----------------------------------------------------------------------------- physics / env
def collide(vn, vt, u, omega, e, mu, m, R):
    out = (ctypes.c_double * 3)()
    lib().or_collide(vn, vt, u, omega, e, mu, m, R, out)
    return out[0], out[1], out[2]


class MT:
    """CPython-compatible `random` stream (random.seed(n) / random() / uniform / randint)."""

    def __init__(self, seed):
        self.s = OrMT()
        lib().or_mt_seed(ctypes.byref(self.s), seed)

    def random(self):
        return lib().or_mt_random(ctypes.byref(self.s))

    def randbelow(self, n):
        return lib().or_mt_randbelow(ctypes.byref(self.s), n)

    def reset_draws(self, params):
        out = (ctypes.c_double * 3)()
        lib().or_reset_draws(ctypes.byref(self.s), ctypes.byref(params), out)
        return out[0], out[1], out[2]


def new_arena(vx, vy, spin):
    a = OrArena()
    lib().or_reset_apply(ctypes.byref(a), vx, vy, spin)
    return a


def arena_state(a):
    return np.array([a.x, a.y, a.vx, a.vy, a.spin, a.top, a.bot, a.scoreA, a.scoreB, a.bounces], np.float64)


def arena_from_state(st):
    a = OrArena()
    a.x, a.y, a.vx, a.vy, a.spin, a.top, a.bot = [float(v) for v in st[:7]]
    a.scoreA, a.scoreB, a.bounces = [int(v) for v in st[7:10]]
    return a


def arena_obs(a):
    oa = np.zeros(7, np.float32)
    ob = np.zeros(7, np.float32)
    lib().or_obs(ctypes.byref(a), oa.ctypes.data, ob.ctypes.data)
    return oa, ob


def step(params, a, aA, aB):
    r = np.zeros(2, np.float32)
    d = lib().or_step(ctypes.byref(params), ctypes.byref(a), int(aA), int(aB), r.ctypes.data)
    oa, ob = arena_obs(a)
    return oa, ob, r, bool(d)


ARENA_DTYPE = np.dtype([("x", "f8"), ("y", "f8"), ("vx", "f8"), ("vy", "f8"), ("spin", "f8"), ("top", "f8"),
                        ("bot", "f8"), ("scoreA", "i4"), ("scoreB", "i4"), ("bounces", "i4"), ("_pad", "i4")])


def arenas_from_soa(st):
    n = np.asarray(st["x"]).shape[0]
    arr = np.zeros(n, ARENA_DTYPE)
    for k in ("x", "y", "vx", "vy", "spin", "top", "bot", "scoreA", "scoreB", "bounces"):
        arr[k] = st[k]
    return arr


def step_arenas(params, arr, aA, aB):
    """Advance a structured array of arenas (ARENA_DTYPE, C layout of or_arena) one tick, no reset.
    Returns obsA, obsB [n,7] f32, rew [n,2] f32, done [n] u8; updates arr in place."""
    assert arr.dtype == ARENA_DTYPE and arr.flags.c_contiguous and ARENA_DTYPE.itemsize == ctypes.sizeof(OrArena)
    n = arr.shape[0]
    aA = np.ascontiguousarray(aA, np.int8)
    aB = np.ascontiguousarray(aB, np.int8)
    obsA = np.zeros((n, 7), np.float32)
    obsB = np.zeros((n, 7), np.float32)
    rew = np.zeros((n, 2), np.float32)
    done = np.zeros(n, np.uint8)
    lib().or_step_batch(ctypes.byref(params), arr.ctypes.data, aA.ctypes.data, aB.ctypes.data, obsA.ctypes.data,
                        obsB.ctypes.data, rew.ctypes.data, done.ctypes.data, n)
    return obsA, obsB, rew, done


def obs_of_arenas(arr):
    """_get_obs_for_A/_B (envs/my_pong_env_2p.py:235-257) for a structured array."""
    oA = np.stack([arr["x"], 1.0 - arr["y"], arr["vx"], -arr["vy"], arr["top"], arr["bot"], arr["spin"]], 1)
    oB = np.stack([arr["x"], arr["y"], arr["vx"], arr["vy"], arr["bot"], arr["top"], arr["spin"]], 1)
    return oA.astype(np.float32), oB.astype(np.float32)


def serve_arenas(arr, mask, vx, vy, spin):
    """reset() (:83-114) applied to arr[mask] with serves (vx, vy, spin)."""
    for k, v in (("scoreA", 0), ("scoreB", 0), ("bounces", 0), ("top", 0.5), ("bot", 0.5), ("x", 0.5), ("y", 0.5)):
        arr[k][mask] = v
    arr["vx"][mask], arr["vy"][mask], arr["spin"][mask] = vx, vy, spin


def rollout_random(params, seed, steps):
    ssum = ctypes.c_int64(0)
    ep = lib().or_rollout_random(ctypes.byref(params), seed, steps, ctypes.byref(ssum))
    return ep, ssum.value


# ----------------------------------------------------------------------------- QNet (numpy)
def scale_noise(raw):
    """models/qnet.py:35-36: x.sign() * sqrt(|x|) (the root correctly rounded, as the device's
    pm_dev.h scale_noise: float(sqrt(double(|x|))))."""
    raw = np.asarray(raw, np.float32)
    sgn = np.where(raw > 0, np.float32(1), np.where(raw < 0, np.float32(-1), np.float32(0))).astype(np.float32)
    return (sgn * np.sqrt(np.abs(raw).astype(np.float64)).astype(np.float32)).astype(np.float32)


def noise_from_raw(raw_in, raw_out):
    """models/qnet.py:37-41 -> (weight_epsilon = outer(f(out), f(in)), bias_epsilon = f(out))."""
    ei, eo = scale_noise(raw_in), scale_noise(raw_out)
    return np.outer(eo, ei).astype(np.float32), eo


def qnet_effective(sd, noisy, eps=None):
    """Fold a QNet state_dict into the effective weights the forward uses (models/qnet.py:43-50).
    noisy=True is train mode: W = mu + sigma*eps (eps from `eps` dict or the state_dict buffers)."""
    g = lambda k: np.asarray(sd[k], np.float64)  # noqa: E731
    out = {"W1": g("features.0.weight"), "b1": g("features.0.bias"),
           "W2": g("features.2.weight"), "b2": g("features.2.bias")}
    for h in ("fc_V", "fc_A"):
        W, b = g(f"{h}.weight_mu"), g(f"{h}.bias_mu")
        if noisy:
            we = np.asarray((eps or sd)[f"{h}.weight_epsilon"], np.float64)
            be = np.asarray((eps or sd)[f"{h}.bias_epsilon"], np.float64)
            # torch evaluates mu + sigma*eps in float32
            W = (np.float32(1) * (np.asarray(sd[f"{h}.weight_mu"], np.float32) +
                                  np.asarray(sd[f"{h}.weight_sigma"], np.float32) * we.astype(np.float32))).astype(np.float64)
            b = (np.asarray(sd[f"{h}.bias_mu"], np.float32) +
                 np.asarray(sd[f"{h}.bias_sigma"], np.float32) * be.astype(np.float32)).astype(np.float64)
        out[h + ".W"], out[h + ".b"] = W, b
    return out


def qnet_features(eff, x):
    x = np.asarray(x, np.float64)
    h1 = np.maximum(x @ eff["W1"].T + eff["b1"], 0.0)
    return np.maximum(h1 @ eff["W2"].T + eff["b2"], 0.0)


def qnet_heads(eff, h):
    V = h @ eff["fc_V.W"].T + eff["fc_V.b"]
    A = h @ eff["fc_A.W"].T + eff["fc_A.b"]
    return V + (A - A.mean(axis=1, keepdims=True))


def qnet_forward(eff, x):
    """QNet.forward (models/qnet.py:71-75), float64."""
    return qnet_heads(eff, qnet_features(eff, x))


def qnet_forward_f32(w, x, want_feat=False):
    """QNet.forward in float32 in the one fixed order libpongmi's matrix-core tile uses (k-ordered
    fmaf chains; oracle/pong_oracle.c or_qnet_f32 states the order). w: an effective-weight block
    (include/pongmi.h PM_QNET_NW floats, plain part first), x [n,7] f32. Returns q [n,3] f32 (and the
    pre-ReLU layer-2 features [n,64] with want_feat). Exact: the device's Q must equal it bitwise."""
    w = np.ascontiguousarray(np.asarray(w, np.float32).ravel()[:4932])
    x = np.ascontiguousarray(x, np.float32).reshape(-1, 7)
    n = x.shape[0]
    q = np.zeros((n, 3), np.float32)
    feat = np.zeros((n, 64), np.float32) if want_feat else None
    lib().or_qnet_f32(w.ctypes.data, x.ctypes.data, n, q.ctypes.data, feat.ctypes.data if want_feat else None)
    return (q, feat) if want_feat else q


def fold_heads_f32(sd, mode):
    """NoisyLinear.forward's effective heads (models/qnet.py:43-50) in torch's float32 arithmetic:
    eval W = mu, train W = mu + (sigma * eps) (product rounded, then the sum). Returns the 4932-float
    plain effective-weight block (W1 | b1 | W2 | b2 | Wh[V, A0..2] | bh)."""
    f = lambda k: np.asarray(sd[k], np.float32)  # noqa: E731
    parts = [f("features.0.weight").ravel(), f("features.0.bias"), f("features.2.weight").ravel(), f("features.2.bias")]
    wh, bh = [], []
    for h in ("fc_V", "fc_A"):
        W, b = f(f"{h}.weight_mu"), f(f"{h}.bias_mu")
        if mode == "train":
            W = W + f(f"{h}.weight_sigma") * f(f"{h}.weight_epsilon")
            b = b + f(f"{h}.bias_sigma") * f(f"{h}.bias_epsilon")
        wh.append(W.reshape(-1, 64))
        bh.append(b.ravel())
    return np.concatenate(parts + [np.concatenate(wh).ravel(), np.concatenate(bh)]).astype(np.float32)


def argmax_first(q):
    """torch argmax: first index of the maximum."""
    return np.argmax(q, axis=1)


# ----------------------------------------------------------------------------- QNetRNN (numpy)
def _sigmoid(x):
    return 0.5 * (1.0 + np.tanh(0.5 * np.asarray(x)))  # = 1 / (1 + e^-x), no overflow


def rnn_effective(sd, train):
    """QNetRNN weights as its forward uses them (models/qnet_rnn.py:43-50, 107-144): NoisyLinear
    layers folded mu + sigma*eps (train mode, torch float32 arithmetic) or mu (eval)."""
    g = lambda k: np.asarray(sd[k], np.float64)  # noqa: E731
    out = {"W1": g("features_extractor.0.weight"), "b1": g("features_extractor.0.bias"),
           "W2": g("features_extractor.2.weight"), "b2": g("features_extractor.2.bias"),
           "Wih": g("lstm.weight_ih_l0"), "Whh": g("lstm.weight_hh_l0"),
           "bih": g("lstm.bias_ih_l0"), "bhh": g("lstm.bias_hh_l0")}
    for name, key in (("S", "fc_shared_head.0"), ("V", "fc_V"), ("A", "fc_A")):
        W, b = np.asarray(sd[f"{key}.weight_mu"], np.float32), np.asarray(sd[f"{key}.bias_mu"], np.float32)
        if train:
            W = W + np.asarray(sd[f"{key}.weight_sigma"], np.float32) * np.asarray(sd[f"{key}.weight_epsilon"], np.float32)
            b = b + np.asarray(sd[f"{key}.bias_sigma"], np.float32) * np.asarray(sd[f"{key}.bias_epsilon"], np.float32)
        out[name + ".W"], out[name + ".b"] = W.astype(np.float64), b.astype(np.float64)
    return out


def rnn_cell(eff, x, h, c):
    """features_extractor + one LSTM step (torch gate order i, f, g, o), float64. x [B,7], h/c [B,128]."""
    f1 = np.maximum(x @ eff["W1"].T + eff["b1"], 0.0)
    f2 = np.maximum(f1 @ eff["W2"].T + eff["b2"], 0.0)
    gates = f2 @ eff["Wih"].T + eff["bih"] + h @ eff["Whh"].T + eff["bhh"]
    i, f, gg, o = np.split(gates, 4, axis=1)
    c2 = _sigmoid(f) * c + _sigmoid(i) * np.tanh(gg)
    h2 = _sigmoid(o) * np.tanh(c2)
    return h2, c2


def rnn_head(eff, h):
    """fc_shared_head (Noisy + ReLU) and the dueling heads: Q = V + (A - mean A)."""
    s = np.maximum(h @ eff["S.W"].T + eff["S.b"], 0.0)
    V = s @ eff["V.W"].T + eff["V.b"]
    A = s @ eff["A.W"].T + eff["A.b"]
    return V + (A - A.mean(axis=1, keepdims=True))


def rnn_forward(eff, xseq, h0, c0):
    """QNetRNN.forward (models/qnet_rnn.py:107-144): xseq [B,T,7], h0/c0 [B,128] -> (q [B,3] of the
    last step, h_T, c_T)."""
    h, c = np.asarray(h0, np.float64), np.asarray(c0, np.float64)
    xseq = np.asarray(xseq, np.float64)
    for t in range(xseq.shape[1]):
        h, c = rnn_cell(eff, xseq[:, t], h, c)
    return rnn_head(eff, h), h, c


RNN_PARAM_KEYS = (  # modelB.parameters() order (models/qnet_rnn.py:71-99)
    "features_extractor.0.weight", "features_extractor.0.bias", "features_extractor.2.weight",
    "features_extractor.2.bias", "lstm.weight_ih_l0", "lstm.weight_hh_l0", "lstm.bias_ih_l0", "lstm.bias_hh_l0") + tuple(
    f"{m}.{s}" for m in ("fc_shared_head.0", "fc_V", "fc_A") for s in ("weight_mu", "bias_mu", "weight_sigma", "bias_sigma"))


def drqn_grads(sd, target_sd, obs, act, rew, nxt, done, gamma=0.99):
    """train_step_rnn's loss and gradients (scripts/train_rnn_iterative.py:424-513), float64: zero
    initial state; q = Q_B(obs)[last step][a_last]; a* = argmax Q_B(next) (first max); y = r_last +
    gamma * Q_T(next)[a*] * (1 - done_last) with targetB in eval mode; loss = smooth_l1(q, y) (beta 1,
    mean); gradients of every modelB parameter by hand-written BPTT (NoisyLinear: d mu = dW,
    d sigma = dW * eps). obs/next [B,T,7], act/rew/done [B,T]. Returns dict(loss, q, y, grads)."""
    eB = rnn_effective(sd, True)
    eT = rnn_effective(target_sd, False)
    B, T, _ = obs.shape
    z = np.zeros((B, 128))
    qn = rnn_forward(eB, nxt, z, z)[0]
    qt = rnn_forward(eT, nxt, z, z)[0]
    a_star = argmax_first(qn)
    y = rew[:, -1].astype(np.float64) + gamma * qt[np.arange(B), a_star] * (~done[:, -1].astype(bool))
    # forward with caches
    x = np.asarray(obs, np.float64)
    f1s, f2s, gs, cs, hs = [], [], [], [z], [z]
    for t in range(T):
        f1 = np.maximum(x[:, t] @ eB["W1"].T + eB["b1"], 0.0)
        f2 = np.maximum(f1 @ eB["W2"].T + eB["b2"], 0.0)
        zt = f2 @ eB["Wih"].T + eB["bih"] + hs[-1] @ eB["Whh"].T + eB["bhh"]
        i, f, g, o = np.split(zt, 4, axis=1)
        i, f, g, o = _sigmoid(i), _sigmoid(f), np.tanh(g), _sigmoid(o)
        c = f * cs[-1] + i * g
        h = o * np.tanh(c)
        f1s.append(f1); f2s.append(f2); gs.append((i, f, g, o)); cs.append(c); hs.append(h)
    hT = hs[-1]
    spre = hT @ eB["S.W"].T + eB["S.b"]
    s = np.maximum(spre, 0.0)
    V = s @ eB["V.W"].T + eB["V.b"]
    A = s @ eB["A.W"].T + eB["A.b"]
    Q = V + (A - A.mean(axis=1, keepdims=True))
    a = np.asarray(act[:, -1], np.int64)
    q = Q[np.arange(B), a]
    d = q - y
    ad = np.abs(d)
    loss = np.mean(np.where(ad < 1.0, 0.5 * d * d, ad - 0.5))
    gq = np.clip(d, -1.0, 1.0) / B
    dQ = np.zeros((B, 3))
    dQ[np.arange(B), a] = gq
    dV = dQ.sum(axis=1, keepdims=True)
    dA = dQ - dQ.sum(axis=1, keepdims=True) / 3.0
    G = {"V.W": dV.T @ s, "V.b": dV.sum(0), "A.W": dA.T @ s, "A.b": dA.sum(0)}
    ds = (dV @ eB["V.W"] + dA @ eB["A.W"]) * (spre > 0)
    G["S.W"], G["S.b"] = ds.T @ hT, ds.sum(0)
    dh = ds @ eB["S.W"]
    dc = np.zeros_like(dh)
    for k in ("Wih", "Whh", "b", "W2", "b2", "W1", "b1"):
        G[k] = 0.0
    for t in range(T - 1, -1, -1):
        i, f, g, o = gs[t]
        tc = np.tanh(cs[t + 1])
        do = dh * tc
        dc = dc + dh * o * (1.0 - tc * tc)
        dzi, dzf, dzg = dc * g * i * (1.0 - i), dc * cs[t] * f * (1.0 - f), dc * i * (1.0 - g * g)
        dzo = do * o * (1.0 - o)
        dz = np.concatenate([dzi, dzf, dzg, dzo], axis=1)
        dc = dc * f
        G["Wih"] = G["Wih"] + dz.T @ f2s[t]
        G["Whh"] = G["Whh"] + dz.T @ hs[t]
        G["b"] = G["b"] + dz.sum(0)
        dh = dz @ eB["Whh"]
        dp2 = (dz @ eB["Wih"]) * (f2s[t] > 0)
        G["W2"] = G["W2"] + dp2.T @ f1s[t]
        G["b2"] = G["b2"] + dp2.sum(0)
        dp1 = (dp2 @ eB["W2"]) * (f1s[t] > 0)
        G["W1"] = G["W1"] + dp1.T @ x[:, t]
        G["b1"] = G["b1"] + dp1.sum(0)
    eps = lambda k: np.asarray(sd[k], np.float64)  # noqa: E731
    grads = {"features_extractor.0.weight": G["W1"], "features_extractor.0.bias": G["b1"],
             "features_extractor.2.weight": G["W2"], "features_extractor.2.bias": G["b2"],
             "lstm.weight_ih_l0": G["Wih"], "lstm.weight_hh_l0": G["Whh"],
             "lstm.bias_ih_l0": G["b"], "lstm.bias_hh_l0": G["b"].copy()}
    for name, key in (("S", "fc_shared_head.0"), ("V", "fc_V"), ("A", "fc_A")):
        grads[f"{key}.weight_mu"] = G[name + ".W"]
        grads[f"{key}.bias_mu"] = G[name + ".b"]
        grads[f"{key}.weight_sigma"] = G[name + ".W"] * eps(f"{key}.weight_epsilon")
        grads[f"{key}.bias_sigma"] = G[name + ".b"] * eps(f"{key}.bias_epsilon")
    return dict(loss=loss, q=q, y=y, grads=grads)


def clip_grad_norm(grads, max_norm=1.0):
    """torch.nn.utils.clip_grad_norm_ (L2 over all tensors): scale by min(1, max_norm / (norm + 1e-6));
    returns (clipped grads, the pre-clip total norm)."""
    norm = float(np.sqrt(sum(float(np.sum(np.square(g))) for g in grads.values())))
    coef = min(1.0, max_norm / (norm + 1e-6))
    return {k: g * coef for k, g in grads.items()}, norm


def drqn_update(sd, target_sd, adam, step, batch, lr=1e-4, gamma=0.99, max_norm=1.0):
    """One train_step_rnn (:400-531): grads, clip_grad_norm_(1.0), Adam(lr) on every modelB
    parameter. adam: {name: (m, v)} (updated in place); step: the Adam step count after this update.
    Returns (new state_dict, info)."""
    info = drqn_grads(sd, target_sd, *batch, gamma=gamma)
    grads, norm = clip_grad_norm(info["grads"], max_norm)
    new = dict(sd)
    for k in RNN_PARAM_KEYS:
        m, v = adam.get(k, (np.zeros_like(grads[k]), np.zeros_like(grads[k])))
        p, m, v = adam_step(np.asarray(sd[k], np.float64), grads[k], m, v, step, lr)
        adam[k] = (m, v)
        new[k] = p
    info["norm"] = norm
    return new, info


def clip_adam_f32(p, m, v, g, norm, at, lr=1e-4, b1=0.9, b2=0.999, eps=1e-8, max_norm=1.0):
    """clip_grad_norm_(max_norm) + torch's Adam step (train_rnn_iterative.py:509-516) restated in
    float32 in the device apply's operation order (k_drqn_apply), the clip coefficient from a given
    pre-clip norm: min(1, max_norm / (norm + 1e-6)); m.lerp_(g, 1 - b1); v.mul_(b2).addcmul_(g, g, 1 - b2);
    p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps). Returns (p, m, v, coef)."""
    f = np.float32
    coef = f(max_norm / (np.float64(f(norm)) + 1e-6))
    coef = min(coef, f(1.0))
    bc1, bc2 = 1.0 - b1 ** at, 1.0 - b2 ** at
    step_size, bc2s = f(lr / bc1), f(np.sqrt(bc2))
    gc = np.asarray(g, f) * coef
    m = np.asarray(m, f) + f(1.0 - b1) * (gc - np.asarray(m, f))
    v = np.asarray(v, f) * f(b2) + f(1.0 - b2) * gc * gc
    denom = np.sqrt(v) / bc2s + f(eps)
    return np.asarray(p, f) - step_size * (m / denom), m, v, coef


def drqn_sigma_map(layout):
    """For the packed QNetRNN block (`layout` = [(key, shape)] in block order, pongmi.rnn.PARAM_LAYOUT):
    (sigma offsets, their mu offsets, their epsilon offsets), one entry per NoisyLinear sigma element."""
    off, o = {}, 0
    for k, s in layout:
        off[k] = (o, int(np.prod(s)))
        o += int(np.prod(s))
    sig, mu, ep = [], [], []
    for k, (o0, n) in off.items():
        if k.endswith("_sigma"):
            base = k[:-len("_sigma")]
            sig.append(np.arange(o0, o0 + n))
            mu.append(np.arange(off[base + "_mu"][0], off[base + "_mu"][0] + n))
            ep.append(np.arange(off[base + "_epsilon"][0], off[base + "_epsilon"][0] + n))
    return np.concatenate(sig), np.concatenate(mu), np.concatenate(ep)


def drqn_apply_packed_f32(params, m, v, gbuf, steps, adam_t, layout, nparam, lr=1e-4, max_norm=1.0, interval=2000,
                          target=None):
    """The sharded DRQN apply (k_drqn_apply, after the all-reduce of the packed exchange buffer
    `gbuf` = [nparam gradients (sigma slots 0) | contributing ranks | void count | ...]) restated in
    float32 on packed blocks: no contributing rank -> nothing; a void count -> nothing (status 8);
    else sigma gradient = summed mu gradient x epsilon, g = grad x (1 / ranks), the norm of that
    global g (float64 sum of squares), clip + Adam (clip_adam_f32), the target copied every
    `interval` steps. Returns dict(params, m, v, target, steps, adam_t, status, norm, coef, g)."""
    f = np.float32
    p, m, v = np.array(params, f), np.array(m, f), np.array(v, f)
    tgt = None if target is None else np.array(target, f)
    ranks = f(gbuf[nparam])
    out = dict(params=p, m=m, v=v, target=tgt, steps=steps, adam_t=adam_t, status=0, norm=None, coef=None, g=None)
    if not ranks > 0:
        return out
    if f(gbuf[nparam + 1]) != 0:
        out["status"] = 8
        return out
    graw = np.array(gbuf[:nparam], f)
    sig, mu, ep = drqn_sigma_map(layout)
    graw[sig] = graw[mu] * p[ep]
    g = graw * (f(1.0) / ranks)
    norm = f(np.sqrt(np.sum(g.astype(np.float64) ** 2)))
    at, ts = adam_t + 1, steps + 1
    p2, m2, v2, coef = clip_adam_f32(p[:nparam], m, v, g, norm, at, lr=lr, max_norm=max_norm)
    p[:nparam] = p2
    if tgt is not None and ts % interval == 0:
        tgt[:] = p
    out.update(params=p, m=m2, v=v2, target=tgt, steps=ts, adam_t=at, norm=norm, coef=coef, g=g)
    return out


# ----------------------------------------------------------------------------- PER (numpy)
def per_sample(prios, size, bs, beta, uniforms, alpha=0.6):
    """PrioritizedReplay.sample (scripts/train_iterative.py:64-73) with np.random.choice's own
    algorithm (cdf = cumsum(p) in float64, cdf /= cdf[-1], searchsorted(u, 'right')) on given uniforms."""
    pr = np.asarray(prios[:size], np.float32)
    probs = pr ** np.float32(alpha)
    probs /= probs.sum()
    cdf = probs.astype(np.float64).cumsum()
    cdf /= cdf[-1]
    idxs = cdf.searchsorted(np.asarray(uniforms, np.float64), side="right")
    w = (np.float32(size) * probs[idxs]) ** np.float32(-beta)
    w = w / w.max()
    return idxs.astype(np.int64), w.astype(np.float32)


# PrioritizedReplay.sample's proportional draw as libpongmi's sum tree evaluates it. np.random.choice
# (:66) normalises p in float32 and searches a float64 cumsum; the device descends fp64 node sums.
# Both pick "the first entry whose running sum of p exceeds u" — the same distribution — but their
# roundings differ near a CDF boundary, so an exact comparison needs the device's own summation
# order. These two functions restate it (csrc/pm_per.h: per_quarter / per_combine / per_chunk_sum
# for the nodes, per_round_prefix / per_lds_search / per_group_find for the descent), from the
# priorities alone; tests/test_gpu_selfplay.py asserts equality for every draw, and
# per_boundary_band() below ties the draw back to np.random.choice's own algorithm.
PER_SUB, PER_FAN, PER_CHUNK = 64, 16, 1024


def _seq_sum(cols):
    """Sequential left-to-right float64 sum over axis 1 (cols [m, k])."""
    acc = np.zeros(cols.shape[0])
    for k in range(cols.shape[1]):
        acc = acc + cols[:, k]
    return acc


_EXP_C = (1.0, 1.0, 0.5, 0.16666666666666666, 0.041666666666666664, 0.008333333333333333, 0.001388888888888889,
          0.0001984126984126984, 2.48015873015873e-05, 2.7557319223985893e-06, 2.755731922398589e-07,
          2.505210838544172e-08, 2.08767569878681e-09, 1.6059043836821613e-10)


def det_pow_f32(p, alpha):
    """csrc/pm_per.h prio_pow restated: the PER leaf prio ** alpha in double from correctly rounded
    operations (atanh-series log, Cody-Waite + Taylor exp), rounded once to float — bit for bit the
    device's leaf, and within an ulp of numpy's float32 power (the reference's, :67)."""
    p = np.asarray(p, np.float32)
    a = np.float64(np.float32(alpha))
    mant, ex = np.frexp(np.where(p > 0, p, np.float32(1)).astype(np.float64))
    m, e = mant * 2.0, ex.astype(np.int64) - 1
    big = m > 1.4142135623730951
    m, e = np.where(big, m * 0.5, m), np.where(big, e + 1, e)
    s = (m - 1.0) / (m + 1.0)
    s2 = s * s
    q = s2 * _horner(s2, _LN_C)
    y = a * (e.astype(np.float64) * 0.69314718055994531 + (2.0 * s + s * q))
    k = np.floor(y * 1.4426950408889634 + 0.5)
    r = (y - k * 6.93147180369123816490e-01) - k * 1.90821492927058770002e-10
    out = np.ldexp(_horner(r, _EXP_C), k.astype(np.int64)).astype(np.float32)
    return np.where(p > 0, out, np.float32(0)).astype(np.float32)


def per_tree(prios, cap, alpha=0.6):
    """Leaves prio_pow(prio, alpha) (f32, det_pow_f32), level-1 nodes ((q0+q1)+q2)+q3 of sequential
    16-leaf fp64 sums, level-2 nodes sequential sums of 16 level-1 nodes. Returns (chunk, sub, leaf)."""
    leaf = det_pow_f32(prios[:cap], alpha)
    nsub = (cap + PER_SUB - 1) // PER_SUB
    nch = (cap + PER_CHUNK - 1) // PER_CHUNK
    lf = np.zeros(nsub * PER_SUB)
    lf[:cap] = leaf.astype(np.float64)
    q = [_seq_sum(lf.reshape(nsub, 4, 16)[:, k, :]) for k in range(4)]
    sub = ((q[0] + q[1]) + q[2]) + q[3]
    sp = np.zeros(nch * PER_FAN)
    sp[:nsub] = sub
    chunk = _seq_sum(sp.reshape(nch, PER_FAN))
    return chunk, sub, leaf


def _wave_incl_scan(v):
    """Hillis-Steele inclusive scan of 64 lanes (v += shfl_up(v, o) for o = 1, 2, .., 32)."""
    v = v.copy()
    for o in (1, 2, 4, 8, 16, 32):
        u = np.concatenate([np.zeros(o), v[:-o]])
        v = np.where(np.arange(64) >= o, v + u, v)
    return v


def _round_prefix(vals):
    """per_round_prefix for one round from base 0: vals [1024] chunk sums -> (incl [1024], total)."""
    v = vals.reshape(256, 4)
    run = np.cumsum(v, axis=1)  # sequential per thread (4 terms: cumsum is left to right)
    acc = run[:, 3]
    incl = np.zeros(1024)
    wsum = []
    for wv in range(4):
        sc = _wave_incl_scan(acc[64 * wv:64 * wv + 64])
        wsum.append(sc[63])
        excl = np.concatenate([[0.0], sc[:-1]])
        wb = 0.0
        for k in range(wv):
            wb = wb + wsum[k]
        ex = wb + excl
        incl[256 * wv:256 * wv + 256] = (ex[:, None] + run[64 * wv:64 * wv + 64]).ravel()
    total = (((0.0 + wsum[0]) + wsum[1]) + wsum[2]) + wsum[3]
    return incl, total


def _group_find(v, x):
    """per_group_find: 4 lanes x NV values in order; first value whose running sum exceeds x, else the
    last nonzero one. Returns (index, sum before it, value)."""
    nv = len(v) // 4
    lanes = v.reshape(4, nv)
    s = [0.0] * 4
    for q in range(4):
        a = 0.0
        for e in range(nv):
            a = a + lanes[q, e]
        s[q] = a
    exs = [0.0, s[0], s[0] + s[1], (s[0] + s[1]) + s[2]]
    hit, nz = None, None
    for q in range(4):
        run = exs[q]
        h = z = None
        for e in range(nv):
            val = lanes[q, e]
            if h is None and run + val > x:
                h = (e, run, val)
            if val > 0.0:
                z = (e, run, val)
            run = run + val
        if h is not None and hit is None:
            hit = (q, h)
        if z is not None:
            nz = (q, z)
    if hit is not None:
        q, (e, b, val) = hit
    elif nz is not None:
        q, (e, b, val) = nz
    else:
        q, (e, b, val) = 0, (0, exs[0], 0.0)
    return q * nv + e, b, val


def per_sample_tree(prios, size, cap, beta, uniforms, alpha=0.6, tree=None):
    """The device's draw (csrc/pm_per.h per_sample_block) for capacities <= 1M (one prefix round):
    indices and un-normalised IS weights (size * P(i))^-beta, exactly as libpongmi computes them.
    prios: the priorities the sample sees (pushes applied). Returns (idx int64, w f32)."""
    chunk, sub, leaf = tree if tree is not None else per_tree(prios, cap, alpha)
    nch = chunk.shape[0]
    assert nch <= 1024, "one prefix round"
    nb = (size + PER_CHUNK - 1) // PER_CHUNK
    vals = np.zeros(1024)
    vals[:nb] = chunk[:nb]
    incl, total = _round_prefix(vals)
    idx = np.zeros(len(uniforms), np.int64)
    w = np.zeros(len(uniforms), np.float32)
    lf = np.asarray(leaf, np.float32)
    for j, u in enumerate(np.asarray(uniforms, np.float64)):
        x = u * total
        k = int(np.searchsorted(incl[:nb] > x, True)) if np.any(incl[:nb] > x) else nb
        if k < nb:
            blk, before = k, (incl[k - 1] if k else 0.0)
        else:
            lo = int(np.argmax(incl[:nb] >= incl[nb - 1]))
            blk, before = lo, (incl[lo - 1] if lo else 0.0)
        sv = np.array([sub[blk * 16 + e] if blk * 16 + e < sub.shape[0] else 0.0 for e in range(16)])
        f1, b1, _ = _group_find(sv, x - before)
        sb = blk * 16 + f1
        e0 = sb * PER_SUB
        lv = np.array([float(lf[e0 + e]) if e0 + e < size else 0.0 for e in range(64)])
        f0, _, pa = _group_find(lv, (x - before) - b1)
        idx[j] = e0 + f0
        w[j] = np.float32(((float(size) * (pa / total)) ** (-beta)))
    return idx, w


def per_boundary_band(prios, size, uniforms, alpha=0.6, tol=5e-7):
    """Which draws lie within `tol` of a CDF boundary of P(i) = prio_i^alpha / sum, where
    np.random.choice's float32-normalised CDF (per_sample) and any exact-order sum may disagree:
    the float32 normalisation moves each CDF value by <= 2^-23 relative, and a 1-ulp difference in a
    float32 prio^alpha moves it by as much again, so 5e-7 bounds the disagreement. Returns a bool mask;
    outside it every correct sampler must pick np.random.choice's index."""
    p = np.asarray(prios[:size], np.float32).astype(np.float64) ** alpha
    cdf = np.cumsum(p) / p.sum()
    u = np.asarray(uniforms, np.float64)
    return np.searchsorted(cdf, u - tol, side="right") != np.searchsorted(cdf, u + tol, side="right")


def per_update(prios, idxs, errors):
    """update_priorities (:74-76): sequential, so the last duplicate wins."""
    for i, e in zip(idxs, errors):
        prios[i] = np.float32(abs(e)) + np.float32(1e-6)


# ----------------------------------------------------------------------------- DQN (numpy)
HEAD_LAYOUT = [("fc_V.weight_mu", (1, 64)), ("fc_V.bias_mu", (1,)), ("fc_V.weight_sigma", (1, 64)),
               ("fc_V.bias_sigma", (1,)), ("fc_A.weight_mu", (3, 64)), ("fc_A.bias_mu", (3,)),
               ("fc_A.weight_sigma", (3, 64)), ("fc_A.bias_sigma", (3,))]
N_HEAD = sum(int(np.prod(s)) for _, s in HEAD_LAYOUT)  # 520


def pack_heads(sd):
    return np.concatenate([np.asarray(sd[k], np.float64).ravel() for k, _ in HEAD_LAYOUT])


def unpack_heads(vec):
    out, o = {}, 0
    for k, s in HEAD_LAYOUT:
        n = int(np.prod(s))
        out[k] = np.asarray(vec[o:o + n]).reshape(s)
        o += n
    return out


def dqn_loss_grads(sdB, heads, target_heads, epsB, s, a, r, ns, d, iw, gamma):
    """Double-DQN loss and head gradients (scripts/train_iterative.py:152-163), float64.
    heads/target_heads: packed 520-vectors (HEAD_LAYOUT). epsB: noise buffers for modelB.
    targetB is in eval mode (train_iterative.py:100) so it uses mu only."""
    hd = unpack_heads(heads)
    th = unpack_heads(target_heads)
    W1 = np.asarray(sdB["features.0.weight"], np.float64)
    feat = {"W1": W1, "b1": np.asarray(sdB["features.0.bias"], np.float64),
            "W2": np.asarray(sdB["features.2.weight"], np.float64), "b2": np.asarray(sdB["features.2.bias"], np.float64)}
    wV_eps = np.asarray(epsB["fc_V.weight_epsilon"], np.float64)
    bV_eps = np.asarray(epsB["fc_V.bias_epsilon"], np.float64)
    wA_eps = np.asarray(epsB["fc_A.weight_epsilon"], np.float64)
    bA_eps = np.asarray(epsB["fc_A.bias_epsilon"], np.float64)
    eff = dict(feat)
    eff["fc_V.W"] = hd["fc_V.weight_mu"] + hd["fc_V.weight_sigma"] * wV_eps
    eff["fc_V.b"] = hd["fc_V.bias_mu"] + hd["fc_V.bias_sigma"] * bV_eps
    eff["fc_A.W"] = hd["fc_A.weight_mu"] + hd["fc_A.weight_sigma"] * wA_eps
    eff["fc_A.b"] = hd["fc_A.bias_mu"] + hd["fc_A.bias_sigma"] * bA_eps
    teff = dict(feat)
    teff["fc_V.W"], teff["fc_V.b"] = th["fc_V.weight_mu"], th["fc_V.bias_mu"]
    teff["fc_A.W"], teff["fc_A.b"] = th["fc_A.weight_mu"], th["fc_A.bias_mu"]
    hs = qnet_features(feat, s)
    hn = qnet_features(feat, ns)
    Qs = qnet_heads(eff, hs)
    B = len(a)
    q = Qs[np.arange(B), a]
    na = argmax_first(qnet_heads(eff, hn))
    nq = qnet_heads(teff, hn)[np.arange(B), na]
    t = np.asarray(r, np.float64) + gamma * nq * (~np.asarray(d, bool))
    diff = q - t
    iw = np.asarray(iw, np.float64)
    loss = np.mean(iw * diff ** 2)
    g = 2.0 * iw * diff / B                       # dL/dq
    gA = np.zeros((B, 3))
    gA[np.arange(B), a] = 1.0
    gA = (gA - 1.0 / 3.0) * g[:, None]            # dL/dA_k
    gV = g[:, None]                               # dL/dV
    dWV = gV.T @ hs                               # [1,64]
    dbV = gV.sum(0)
    dWA = gA.T @ hs                               # [3,64]
    dbA = gA.sum(0)
    grads = {"fc_V.weight_mu": dWV, "fc_V.bias_mu": dbV, "fc_V.weight_sigma": dWV * wV_eps,
             "fc_V.bias_sigma": dbV * bV_eps, "fc_A.weight_mu": dWA, "fc_A.bias_mu": dbA,
             "fc_A.weight_sigma": dWA * wA_eps, "fc_A.bias_sigma": dbA * bA_eps}
    gvec = np.concatenate([grads[k].ravel() for k, _ in HEAD_LAYOUT])
    return dict(loss=loss, q=q, targets=t, na=na, errors=np.abs(diff), grads=gvec)


def adam_step(p, g, m, v, t, lr, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch.optim.Adam single-tensor update (no weight decay, no amsgrad), step t >= 1."""
    m = m + (1 - beta1) * (g - m)                 # exp_avg.lerp_(grad, 1-beta1)
    v = v * beta2 + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** t
    bc2 = 1 - beta2 ** t
    denom = np.sqrt(v) / np.sqrt(bc2) + eps
    p = p - (lr / bc1) * (m / denom)
    return p, m, v


# ----------------------------------------------------------------------------- Philox (numpy)
# Restatement of the counter-based generator libpongmi draws from (Philox4x32-10, Salmon et al.
# SC'11), so tests can replay the device's serves / epsilon draws / PER uniforms / noise.
TAG_SERVE, TAG_ACT, TAG_OPP, TAG_NOISE_ACT, TAG_PER, TAG_NOISE_TRAIN = 1, 2, 3, 4, 5, 6
TAG_SERVE_STEP = 9
_M0, _M1, _W0, _W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85


def philox(c0, c1, c2, c3, key):
    """Vectorised Philox4x32-10 over uint32 arrays; key is a 64-bit int."""
    m32 = np.uint64(0xFFFFFFFF)
    c = [np.asarray(v, np.uint64) & m32 for v in (c0, c1, c2, c3)]
    k0, k1 = np.uint64(key & 0xFFFFFFFF), np.uint64((key >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = c[0] * np.uint64(_M0)
        p1 = c[2] * np.uint64(_M1)
        hi0, lo0 = p0 >> np.uint64(32), p0 & m32
        hi1, lo1 = p1 >> np.uint64(32), p1 & m32
        c = [(hi1 ^ c[1] ^ k0) & m32, lo1, (hi0 ^ c[3] ^ k1) & m32, lo0]
        k0 = (k0 + np.uint64(_W0)) & m32
        k1 = (k1 + np.uint64(_W1)) & m32
    return [v.astype(np.uint32) for v in c]


def philox64(index, tag, ctr, key):
    ctr = np.asarray(ctr, np.uint64)
    return philox(index, tag, ctr & np.uint64(0xFFFFFFFF), ctr >> np.uint64(32), key)


def u53(hi, lo):
    v = ((np.asarray(hi, np.uint64) << np.uint64(32)) | np.asarray(lo, np.uint64)) >> np.uint64(11)
    return v.astype(np.float64) * 2.0 ** -53


def below(r, n):
    return ((np.asarray(r, np.uint64) * np.uint64(n)) >> np.uint64(32)).astype(np.int64)


# pm_dev.h normal(): Box-Muller's cos branch in double with +, -, *, /, sqrt only, in the device's
# exact evaluation order (numpy float64 elementwise operations are the same correctly rounded IEEE
# operations and never fuse), rounded once to float: bit-identical to every device draw.
_LN_C = (0.66666666666666663, 0.40000000000000002, 0.28571428571428570, 0.22222222222222221, 0.18181818181818182,
         0.15384615384615385, 0.13333333333333333, 0.11764705882352941, 0.10526315789473684, 0.09523809523809523)
_COS_C = (-0.5, 0.041666666666666664, -0.0013888888888888889, 2.4801587301587302e-05, -2.755731922398589e-07,
          2.0876756987868100e-09, -1.1470745597729725e-11)
_SIN_C = (-0.16666666666666666, 0.0083333333333333332, -0.00019841269841269841, 2.7557319223985893e-06,
          -2.5052108385441720e-08, 1.6059043836821613e-10, -7.6471637318198164e-13)


def _horner(z, coefs):
    """c0 + z * (c1 + z * (... + z * c_last)), evaluated innermost first."""
    acc = np.full(np.shape(z), coefs[-1], np.float64)
    for c in coefs[-2::-1]:
        acc = c + z * acc
    return acc


def det_ln_u1(k):
    """pm_dev.h det_ln_u1: ln(k 2^-24) for integer k in [1, 2^24]."""
    mant, ex = np.frexp(np.asarray(k, np.float64))  # k = mant 2^ex, mant in [0.5, 1): m = 2 mant in [1, 2)
    m, e = mant * 2.0, ex.astype(np.int64) - 1
    big = m > 1.4142135623730951
    m, e = np.where(big, m * 0.5, m), np.where(big, e + 1, e)
    s = (m - 1.0) / (m + 1.0)
    s2 = s * s
    p = s2 * _horner(s2, _LN_C)
    return (e - 24).astype(np.float64) * 0.69314718055994531 + (2.0 * s + s * p)


def det_cos_turn(t):
    """pm_dev.h det_cos_turn: cos(2 pi t) for t on the 24-bit grid of [0, 1)."""
    t = np.asarray(t, np.float64)
    q = np.floor(4.0 * t + 0.5)
    th = 6.2831853071795862 * (t - 0.25 * q)
    z = th * th
    c = 1.0 + z * _horner(z, _COS_C)
    sn = th * (1.0 + z * _horner(z, _SIN_C))
    qi = q.astype(np.int64) & 3
    return np.where(qi == 0, c, np.where(qi == 1, -sn, np.where(qi == 2, -c, sn)))


def normal_f32(a, b):
    """The device's N(0, 1) draw (pm_dev.h normal) from two u32 arrays, bit for bit."""
    k = (np.asarray(a, np.uint32) >> 8).astype(np.int64) + 1
    r = np.sqrt(-2.0 * det_ln_u1(k))
    u2 = (np.asarray(b, np.uint32) >> 8).astype(np.float64) * 2.0 ** -24
    return (r * det_cos_turn(u2)).astype(np.float32)


def sincos_serve(x):
    """pm_dev.h sincos_serve restated (numpy float64, same operation order): sin and cos of x for
    |x| < 3 pi / 4 by one Cody-Waite step and fdlibm's __kernel_sin / __kernel_cos, bit for bit."""
    x = np.asarray(x, np.float64)
    pio4, pio2_1, pio2_1t = 7.85398163397448278999e-01, 1.57079632673412561417e+00, 6.07710050650619224932e-11
    n = np.where(x > pio4, 1, np.where(x < -pio4, -1, 0))
    z0 = np.where(n > 0, x - pio2_1, x + pio2_1)
    t = np.where(n > 0, pio2_1t, -pio2_1t)
    y0 = z0 - t
    y1 = (z0 - y0) - t
    y0 = np.where(n == 0, x, y0)
    y1 = np.where(n == 0, 0.0, y1)
    S1, S2, S3 = -1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04
    S4, S5, S6 = 2.75573137070700676789e-06, -2.50507602534068634195e-08, 1.58969099521155010221e-10
    z = y0 * y0
    v = z * y0
    rs = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)))
    ks = y0 - ((z * (0.5 * y1 - v * rs) - y1) - v * S1)
    C1, C2, C3 = 4.16666666666666019037e-02, -1.38888888888741095749e-03, 2.48015872894767294178e-05
    C4, C5, C6 = -2.75573143513906633035e-07, 2.08757232129817482790e-09, -1.13596475577881948265e-11
    rc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))))
    hz = 0.5 * z
    w = 1.0 - hz
    kc = w + (((1.0 - w) - hz) + (z * rc - y0 * y1))
    s = np.where(n == 0, ks, np.where(n > 0, kc, -kc))
    c = np.where(n == 0, kc, np.where(n > 0, -ks, ks))
    return s, c


def philox_serve(params_dict, i, nserve, seed, step=None):
    """The device's production serve (pm_dev.h serve_draw) restated: arrays i, nserve. With `step`
    (K1's step-keyed stream, ABI 15: pm_env_step's counter) the key is (i, TAG_SERVE_STEP, step lo,
    step hi) and nserve is ignored."""
    p = params_dict
    if step is None:
        r0 = philox(i, TAG_SERVE, nserve, 0, seed)
        r1 = philox(i, TAG_SERVE | 0x100, nserve, 0, seed)
    else:
        lo, hi = int(step) & 0xFFFFFFFF, int(step) >> 32
        r0 = philox(i, TAG_SERVE_STEP, lo, hi, seed)
        r1 = philox(i, TAG_SERVE_STEP | 0x100, lo, hi, seed)
    speed = p["speed_lo"] + (p["speed_hi"] - p["speed_lo"]) * u53(r0[0], r0[1])
    coin = u53(r0[2], r0[3]) < 0.5
    u = u53(r1[0], r1[1])
    ang = np.where(coin, p["ang0_lo"] + (p["ang0_hi"] - p["ang0_lo"]) * u, p["ang1_lo"] + (p["ang1_hi"] - p["ang1_lo"]) * u)
    rad = ang * (3.141592653589793 / 180.0)
    spin = p["spin_lo"] + (p["spin_hi"] - p["spin_lo"]) * u53(r1[2], r1[3])
    sn, cs = sincos_serve(rad)
    far = ~(np.abs(rad) < 2.35619449019234483700)  # the device redoes these with OCML's sincos (< 1 ulp)
    sn, cs = np.where(far, np.sin(rad), sn), np.where(far, np.cos(rad), cs)
    return speed * cs, speed * sn, spin


def philox_noise(seed, tag, ctr):
    """Factorised noise of one QNet head pair as the device draws it (pm_dev.h fold_heads):
    returns (fV_in[64], fV_out[1], fA_in[64], fA_out[3]) after scale_noise."""
    out = []
    for layer, (n_in, n_out) in enumerate(((64, 1), (64, 3))):
        for which, n in ((0, n_in), (1, n_out)):
            e = np.arange(n)
            r = philox64(e, tag | (layer << 8) | (which << 12), np.full(n, ctr, np.uint64), seed)
            out.append(scale_noise(normal_f32(r[0], r[1])))
    return out


TAG_NOISE_RNN = 7


def rnn_philox_noise(seed, ctr):
    """QNetRNN's reset_noise (models/qnet_rnn.py:33-41, the three NoisyLinear layers fc_shared_head.0,
    fc_V, fc_A) as the device draws it (pm_rnn.hip rnn_noise: Philox(e, TAG_NOISE_RNN | layer << 8 |
    which << 12, ctr), Box-Muller, _scale_noise), returned as the epsilon buffers reset_noise leaves:
    {key.weight_epsilon: eps_out.ger(eps_in), key.bias_epsilon: eps_out}."""
    out = {}
    for layer, (key, n_in, n_out) in enumerate((("fc_shared_head.0", 128, 128), ("fc_V", 128, 1), ("fc_A", 128, 3))):
        f = []
        for which, n in ((0, n_in), (1, n_out)):
            e = np.arange(n)
            r = philox64(e, TAG_NOISE_RNN | (layer << 8) | (which << 12), np.full(n, ctr, np.uint64), seed)
            f.append(scale_noise(normal_f32(r[0], r[1])))
        out[f"{key}.weight_epsilon"] = np.outer(f[1], f[0]).astype(np.float32)
        out[f"{key}.bias_epsilon"] = f[1]
    return out


def rnn_act_decision(q, eps, seed, ctr, arenas):
    """select_action_for_model's choice (scripts/train_rnn_iterative.py:371-389) — and
    select_action_B's (scripts/train_iterative.py:124-130), the same rule — with the device's Philox
    streams: random.random() < eps ? randint(0, 2) : argmax Q (first max). Returns (action, explore
    mask); eps <= 0 never explores (the opponents' greedy act)."""
    greedy = argmax_first(q)
    if eps <= 0.0:
        return greedy, np.zeros(len(greedy), bool)
    r = philox64(arenas, TAG_ACT, np.full(len(arenas), ctr, np.uint64), seed)
    explore = u53(r[0], r[1]) < eps
    return np.where(explore, below(r[2], 3), greedy), explore


eps_greedy = rnn_act_decision
