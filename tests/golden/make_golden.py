#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run only in the build container (the reference does not exist on the GPU box):

    python -B tests/golden/make_golden.py

The reference's `envs/`, `models/` and the `PrioritizedReplay` class of
`scripts/train_iterative.py` are imported from /root/reference with `gym`, `gym.spaces` and `pygame`
replaced by inert stubs (they are used only as a base class / space descriptors / for rendering:
envs/my_pong_env_2p.py:1-2,40,66,73,75-79,84). Nothing from the reference is copied into the
repository: only inputs and the reference's outputs are written, as .npz data.

Fixtures:
  collide_kat.npz   envs/physics.py:3-23 known-answer table (stick / slide / +-0 vrel / int e)
  env_<cfg>.npz     per-arena PongEnv2P trajectories (envs/my_pong_env_2p.py:83-232), serves drawn
                    from the global `random` stream after random.seed(seed_i)
  rollout_random.npz config-1 loop: random-vs-random with randint actions from the same stream
  qnet.npz          models/qnet.py QNet forward (eval / train mode) on model5-5_fault.pth weights,
                    NoisyLinear.reset_noise transform (models/qnet.py:33-41)
  dqn_steps.npz     three consecutive train_step bodies (scripts/train_iterative.py:141-168)
  per.npz           PrioritizedReplay push / sample / update_priorities (scripts/train_iterative.py:49-76)
"""
import ast
import copy
import os
import random
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
REF = os.environ.get("PONG_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")

    class Env:
        def __init__(self, *a, **k):
            pass

        def reset(self, seed=None, options=None):
            return None

    class MultiDiscrete:
        def __init__(self, nvec):
            self.nvec = np.asarray(nvec)

    class Box:
        def __init__(self, low, high, dtype=None, shape=None):
            self.low, self.high = low, high
            self.shape = np.asarray(low).shape

    gym.Env = Env
    spaces.MultiDiscrete = MultiDiscrete
    spaces.Box = Box
    gym.spaces = spaces
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = spaces
    sys.modules["pygame"] = types.ModuleType("pygame")


_install_stubs()
sys.path.insert(0, REF)
import torch  # noqa: E402
import yaml  # noqa: E402

import envs.my_pong_env_2p as ref_env_mod  # noqa: E402
import envs.physics as ref_phys  # noqa: E402
from models.qnet import QNet, NoisyLinear  # noqa: E402

PARAM_SETS = {}
with open(os.path.join(REF, "config.yaml")) as f:
    PARAM_SETS["cfg"] = yaml.safe_load(f)["env"]
with open(os.path.join(REF, "config_rnn.yaml")) as f:
    PARAM_SETS["rnn"] = yaml.safe_load(f)["env"]
# constructor defaults (envs/my_pong_env_2p.py:19-37): restitution 0.9 < 1, friction 0.2 -> slide-heavy
PARAM_SETS["default"] = {}

STATE_FIELDS = ["ball_x", "ball_y", "ball_vx", "ball_vy", "spin", "top_paddle_x", "bottom_paddle_x",
                "scoreA", "scoreB", "bounce_count"]


def _state(env):
    return np.array([float(getattr(env, k)) for k in STATE_FIELDS], dtype=np.float64)


def _param_record(env):
    ai = env.ball_angle_intervals
    return dict(
        paddle_width=env.paddle_width, paddle_speed=env.paddle_speed, magnus_factor=env.magnus_factor,
        restitution=float(env.restitution), friction=env.friction, ball_mass=env.ball_mass,
        world_ball_radius=env.world_ball_radius,
        speed_lo=env.ball_speed_range[0], speed_hi=env.ball_speed_range[1],
        spin_lo=env.spin_range[0], spin_hi=env.spin_range[1],
        ang0_lo=ai[0][0], ang0_hi=ai[0][1], ang1_lo=ai[1][0], ang1_hi=ai[1][1],
        speed_increment=env.speed_increment, max_score=env.max_score,
        speed_scale_every=env.speed_scale_every, enable_spin=int(bool(env.enable_spin)),
    )


# ------------------------------------------------------------------------- collide KAT
def make_collide():
    rng = np.random.RandomState(1234)
    rows, outs = [], []
    M = 4000
    for i in range(M):
        vn = rng.uniform(-0.08, 0.08)
        vt = rng.uniform(-0.08, 0.08)
        u = [0.0, 0.03, -0.03, 0.02, -0.02][rng.randint(5)]
        om = rng.uniform(-8, 8)
        e = [1, 1.0, 0.9, 0.5][rng.randint(4)]
        mu = [0.6, 0.2, 0.0, 1.5][rng.randint(4)]
        m = [1.0, 2.0, 0.5][rng.randint(3)]
        R = [0.03, 0.05][rng.randint(2)]
        rows.append((vn, vt, u, om, float(e), mu, m, R))
        outs.append(ref_phys.collide_sphere_with_moving_plane(vn, vt, u, om, e, mu, m, R))
    # exact edge cases: vrel = +0.0 / -0.0 on the slide branch, zero vn, int restitution
    R = 0.03
    for (vn, vt, u, om) in [(0.05, 0.0, 0.0, 0.0), (0.05, -0.0, 0.0, 0.0), (0.05, 0.0, -0.0, 0.0),
                            (0.0, 0.01, 0.0, 0.0), (0.04, 0.03, 0.03, 0.0), (-0.04, 0.03, 0.03, -0.0)]:
        for e in (1, 1.0, 0.9):
            rows.append((vn, vt, u, om, float(e), 0.0, 1.0, R))
            outs.append(ref_phys.collide_sphere_with_moving_plane(vn, vt, u, om, e, 0.0, 1.0, R))
    np.savez_compressed(os.path.join(OUT, "collide_kat.npz"),
                        inputs=np.array(rows, dtype=np.float64), outputs=np.array(outs, dtype=np.float64))
    print("collide_kat", len(rows))


# ------------------------------------------------------------------------- env trajectories
def make_env(name, n_arenas=12, steps=320):
    kw = dict(PARAM_SETS[name])
    hits = {"stick": 0, "slide": 0}
    orig = ref_env_mod.collide_sphere_with_moving_plane

    def spy(vn, vt, u, omega, e, mu, m, R):
        jt_star = (2 * m / 7.0) * (u + R * omega - vt)
        hits["stick" if abs(jt_star) <= mu * m * (1 + e) * abs(vn) else "slide"] += 1
        return orig(vn, vt, u, omega, e, mu, m, R)

    ref_env_mod.collide_sphere_with_moving_plane = spy
    seeds = np.array([1000 + 17 * i for i in range(n_arenas)], dtype=np.int64)
    init = np.zeros((n_arenas, 10))
    init_obs = np.zeros((n_arenas, 2, 7), np.float32)
    actA = np.zeros((n_arenas, steps), np.int8)
    actB = np.zeros((n_arenas, steps), np.int8)
    state = np.zeros((n_arenas, steps, 10))
    obsA = np.zeros((n_arenas, steps, 7), np.float32)
    obsB = np.zeros((n_arenas, steps, 7), np.float32)
    rew = np.zeros((n_arenas, steps, 2), np.float32)
    done = np.zeros((n_arenas, steps), np.uint8)
    reset_state = np.full((n_arenas, steps, 10), np.nan)
    reset_obs = np.zeros((n_arenas, steps, 2, 7), np.float32)
    params = None
    for i in range(n_arenas):
        random.seed(int(seeds[i]))
        env = ref_env_mod.PongEnv2P(**kw)
        params = _param_record(env)
        init[i] = _state(env)
        o = env._get_obs()
        init_obs[i, 0], init_obs[i, 1] = o
        pol = np.random.RandomState(int(seeds[i]))
        for t in range(steps):
            acts = []
            for who in (0, 1):
                ob = o[who]
                if pol.rand() < 0.6:  # ball follower with tolerance 0.02 (tests/arena.py:209-215)
                    bx, px = ob[0], ob[4]
                    acts.append(0 if bx < px - 0.02 else (2 if bx > px + 0.02 else 1))
                else:
                    acts.append(int(pol.randint(3)))
            actA[i, t], actB[i, t] = acts
            (nA, nB), (rA, rB), d, _ = env.step(acts[0], acts[1])
            state[i, t] = _state(env)
            obsA[i, t], obsB[i, t] = nA, nB
            rew[i, t] = (rA, rB)
            done[i, t] = d
            if d:
                o = env.reset()
                reset_state[i, t] = _state(env)
                reset_obs[i, t, 0], reset_obs[i, t, 1] = o
            else:
                o = (nA, nB)
    ref_env_mod.collide_sphere_with_moving_plane = orig
    np.savez_compressed(os.path.join(OUT, f"env_{name}.npz"), seeds=seeds, init=init, init_obs=init_obs,
                        actA=actA, actB=actB, state=state, obsA=obsA, obsB=obsB, rew=rew, done=done,
                        reset_state=reset_state, reset_obs=reset_obs,
                        param_names=np.array(list(params.keys())),
                        param_values=np.array([float(v) for v in params.values()]),
                        hits_stick=hits["stick"], hits_slide=hits["slide"])
    print(f"env_{name}: episodes={int(done.sum())} stick={hits['stick']} slide={hits['slide']} "
          f"bounces_max={int(state[..., 9].max())}")


# ------------------------------------------------------------------------- config-1 loop
def make_rollout_random():
    out = {}
    for name in ("cfg", "rnn"):
        random.seed(0)
        env = ref_env_mod.PongEnv2P(**PARAM_SETS[name])
        steps, episodes, ssum = 20000, 0, 0
        for _ in range(steps):
            aA = random.randint(0, 2)
            aB = random.randint(0, 2)
            _, _, d, _ = env.step(aA, aB)
            if d:
                episodes += 1
                ssum += env.scoreA - env.scoreB
                env.reset()
        out[f"{name}_steps"] = steps
        out[f"{name}_episodes"] = episodes
        out[f"{name}_score_sum"] = ssum
        out[f"{name}_final_state"] = _state(env)
    np.savez_compressed(os.path.join(OUT, "rollout_random.npz"), **out)
    print("rollout_random", {k: v for k, v in out.items() if not k.endswith("state")})


# ------------------------------------------------------------------------- QNet
def _sd_to_np(sd, prefix):
    return {f"{prefix}{k}": v.detach().cpu().numpy().astype(np.float32) for k, v in sd.items()}


def _obs_batch(rng, n):
    lo = np.array([0, 0, -0.08, -0.08, 0, 0, -5], np.float32)
    hi = np.array([1, 1, 0.08, 0.08, 1, 1, 5], np.float32)
    return (lo + (hi - lo) * rng.random_sample((n, 7))).astype(np.float32)


def make_qnet():
    cp = torch.load(os.path.join(REF, "checkpoints", "model5-5_fault.pth"), map_location="cpu", weights_only=True)
    rng = np.random.RandomState(7)
    obs = _obs_batch(rng, 256)
    x = torch.from_numpy(obs)
    out = {"obs": obs}
    for who in ("modelB", "modelA"):
        net = QNet(7, 3)
        net.load_state_dict(cp[who], strict=True)
        out.update(_sd_to_np(net.state_dict(), f"{who}."))
        with torch.no_grad():
            net.train()
            out[f"{who}.q_train"] = net(x).numpy()
            net.eval()
            out[f"{who}.q_eval"] = net(x).numpy()
    # NoisyLinear.reset_noise transform: record raw N(0,1) draws and the resulting buffers
    lin = NoisyLinear(64, 3)
    torch.manual_seed(123)
    raw_in = torch.randn(64)
    raw_out = torch.randn(3)
    torch.manual_seed(123)
    lin.reset_noise()
    out["noise.raw_in"] = raw_in.numpy()
    out["noise.raw_out"] = raw_out.numpy()
    out["noise.weight_epsilon"] = lin.weight_epsilon.numpy()
    out["noise.bias_epsilon"] = lin.bias_epsilon.numpy()
    np.savez_compressed(os.path.join(OUT, "qnet.npz"), **out)
    print("qnet", out["modelB.q_train"][:2])


# ------------------------------------------------------------------------- DQN train_step
def make_dqn():
    """Three consecutive train_step bodies, restated from scripts/train_iterative.py:141-168 around
    the reference's own QNet and torch.optim.Adam (lr 2.5e-4: config.yaml:34, gamma 0.99)."""
    cp = torch.load(os.path.join(REF, "checkpoints", "model5-5_fault.pth"), map_location="cpu", weights_only=True)
    modelB = QNet(7, 3)
    modelB.load_state_dict(cp["modelB"], strict=True)
    for p in modelB.features.parameters():
        p.requires_grad = False
    targetB = copy.deepcopy(modelB)
    targetB.eval()
    head_params = list(modelB.fc_V.parameters()) + list(modelB.fc_A.parameters())
    names = [n for n, _ in list(modelB.fc_V.named_parameters(prefix="fc_V")) +
             list(modelB.fc_A.named_parameters(prefix="fc_A"))]
    opt = torch.optim.Adam(head_params, lr=2.5e-4)
    gamma, target_update_interval = 0.99, 2
    out = _sd_to_np(modelB.state_dict(), "init.")
    out["param_names"] = np.array(names)
    rng = np.random.RandomState(11)
    train_steps = 0
    for step in range(3):
        B = 256
        s = _obs_batch(rng, B)
        ns = _obs_batch(rng, B)
        a = rng.randint(0, 3, B).astype(np.int64)
        r = rng.choice([-1.0, 0.0, 0.0, 0.0, 1.0], B).astype(np.float32)
        d = rng.rand(B) < 0.1
        iw = rng.uniform(0.2, 1.0, B).astype(np.float32)
        iw /= iw.max()
        torch.manual_seed(1000 + step)
        modelB.reset_noise()
        targetB.reset_noise()
        out[f"s{step}.s"], out[f"s{step}.ns"], out[f"s{step}.a"] = s, ns, a
        out[f"s{step}.r"], out[f"s{step}.d"], out[f"s{step}.iw"] = r, d, iw
        for k, v in modelB.state_dict().items():
            if "epsilon" in k:
                out[f"s{step}.noiseB.{k}"] = v.numpy().copy()
        st, at, rt, nst, dt = map(torch.from_numpy, (s, a, r, ns, d))
        iwt = torch.from_numpy(iw)
        q_vals = modelB(st).gather(1, at.unsqueeze(1)).squeeze(1)
        with torch.no_grad():
            na = modelB(nst).argmax(1, keepdim=True)
            nq = targetB(nst).gather(1, na).squeeze(1)
        targets = rt + gamma * nq * (~dt)
        loss = (iwt * (q_vals - targets).pow(2)).mean()
        opt.zero_grad()
        loss.backward()
        out[f"s{step}.grads"] = np.concatenate([p.grad.numpy().ravel() for p in head_params])
        opt.step()
        errors = (q_vals - targets).detach().abs().numpy()
        out[f"s{step}.loss"] = np.float32(loss.item())
        out[f"s{step}.q"] = q_vals.detach().numpy()
        out[f"s{step}.targets"] = targets.detach().numpy()
        out[f"s{step}.na"] = na.squeeze(1).numpy()
        out[f"s{step}.errors"] = errors
        out[f"s{step}.params_after"] = np.concatenate([p.detach().numpy().ravel() for p in head_params])
        train_steps += 1
        if train_steps % target_update_interval == 0:
            targetB.load_state_dict(modelB.state_dict())
        out[f"s{step}.target_heads_after"] = np.concatenate(
            [p.detach().numpy().ravel() for p in list(targetB.fc_V.parameters()) + list(targetB.fc_A.parameters())])
    np.savez_compressed(os.path.join(OUT, "dqn_steps.npz"), **out)
    print("dqn", [float(out[f"s{i}.loss"]) for i in range(3)])


# ------------------------------------------------------------------------- PER
def _lift_class(path, cls_name, ns):
    src = open(path).read()
    tree = ast.parse(src)
    node = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls_name)
    mod = ast.Module(body=[node], type_ignores=[])
    exec(compile(mod, path, "exec"), ns)
    return ns[cls_name]


def make_per():
    ns = {"np": np, "torch": torch, "device": "cpu"}
    PR = _lift_class(os.path.join(REF, "scripts", "train_iterative.py"), "PrioritizedReplay", ns)
    rng = np.random.RandomState(5)
    out = {}
    cap = 1000
    per = PR(cap, alpha=0.6)
    phase = 0
    for n_push, n_upd in ((300, 3), (900, 4), (500, 2)):  # not-full, wrap, wrap again
        pushed_max = []
        for i in range(n_push):
            pushed_max.append(per.prios.max() if per.buffer else 1.0)
            per.push((i,))
        out[f"p{phase}.push_max"] = np.array(pushed_max, np.float32)
        out[f"p{phase}.n_push"] = n_push
        for u in range(n_upd):
            beta = 0.4 + 0.15 * u
            seed = 100 * phase + u
            np.random.seed(seed)
            batch, idxs, w = per.sample(64, beta)
            np.random.seed(seed)
            uni = np.random.random_sample(64)
            out[f"p{phase}.u{u}.prios_before"] = per.prios.copy()
            out[f"p{phase}.u{u}.size"] = len(per.buffer)
            out[f"p{phase}.u{u}.pos"] = per.pos
            out[f"p{phase}.u{u}.beta"] = beta
            out[f"p{phase}.u{u}.uniforms"] = uni
            out[f"p{phase}.u{u}.idxs"] = np.asarray(idxs, np.int64)
            out[f"p{phase}.u{u}.weights"] = w.numpy()
            errs = rng.uniform(0, 2, 64).astype(np.float32)
            errs[::7] = errs[3]  # exercise duplicate-index updates too
            upd_idx = np.asarray(idxs).copy()
            upd_idx[1::9] = upd_idx[0]
            per.update_priorities(upd_idx, errs)
            out[f"p{phase}.u{u}.upd_idx"] = upd_idx
            out[f"p{phase}.u{u}.upd_err"] = errs
            out[f"p{phase}.u{u}.prios_after"] = per.prios.copy()
        phase += 1
    out["n_phases"] = phase
    out["cap"] = cap
    np.savez_compressed(os.path.join(OUT, "per.npz"), **out)
    print("per", phase, "phases")


if __name__ == "__main__":
    make_collide()
    for name in PARAM_SETS:
        make_env(name)
    make_rollout_random()
    make_qnet()
    make_dqn()
    make_per()
