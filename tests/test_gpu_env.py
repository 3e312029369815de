"""K1 parity on the device: pm_env_reset / pm_env_step / pm_collide against the reference's own
trajectories (tests/golden, bit-exact) and against the oracle at full batch sizes (bit-exact)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

STATE_ORDER = ("x", "y", "vx", "vy", "spin", "top", "bot", "scoreA", "scoreB", "bounces")


def _kwargs_from_golden(g):
    pv = dict(zip([str(n) for n in g["param_names"]], g["param_values"].tolist()))
    return dict(paddle_width=pv["paddle_width"], paddle_speed=pv["paddle_speed"], max_score=int(pv["max_score"]),
                enable_spin=bool(pv["enable_spin"]), magnus_factor=pv["magnus_factor"],
                restitution=pv["restitution"], friction=pv["friction"], ball_mass=pv["ball_mass"],
                world_ball_radius=pv["world_ball_radius"], ball_speed_range=(pv["speed_lo"], pv["speed_hi"]),
                spin_range=(pv["spin_lo"], pv["spin_hi"]),
                ball_angle_intervals=[[pv["ang0_lo"], pv["ang0_hi"]], [pv["ang1_lo"], pv["ang1_hi"]]],
                speed_scale_every=int(pv["speed_scale_every"]), speed_increment=pv["speed_increment"]), pv


def _state_matrix(env):
    st = env.get_state()
    return np.stack([np.asarray(st[k], np.float64) for k in STATE_ORDER], 1)


@pytest.mark.parametrize("name", ["cfg", "rnn", "default"])
def test_env_matches_reference_trajectories_bit_exact(golden, name):
    """All golden arenas stepped in one batch with the recorded actions; serves drawn host-side
    with CPython's random exactly as the reference (parity mode). Every fp64 state word, obs,
    reward, done and score must be identical at every step, including autoreset serves."""
    from pongmi.env import PongEnv2PBatch, serve_table_from_random

    g = golden(f"env_{name}")
    kw, _ = _kwargs_from_golden(g)
    n, T = g["actA"].shape
    table = serve_table_from_random(g["seeds"], int(g["done"].sum(1).max()) + 1, **kw)
    env = PongEnv2PBatch(n, seed=0, serve_table=table, autoreset=True, **kw)
    oA, oB = env.reset()
    assert np.array_equal(_state_matrix(env), g["init"])
    assert np.array_equal(oA.cpu().numpy(), g["init_obs"][:, 0]) and np.array_equal(oB.cpu().numpy(), g["init_obs"][:, 1])
    for t in range(T):
        (oA, oB), (rA, rB), done, info = env.step(torch.from_numpy(g["actA"][:, t]), torch.from_numpy(g["actB"][:, t]))
        d = done.cpu().numpy().astype(bool)
        assert np.array_equal(d, g["done"][:, t].astype(bool)), t
        assert np.array_equal(rA.cpu().numpy(), g["rew"][:, t, 0]) and np.array_equal(rB.cpu().numpy(), g["rew"][:, t, 1])
        assert np.array_equal(info["term_obsA"].cpu().numpy(), g["obsA"][:, t])
        assert np.array_equal(info["term_obsB"].cpu().numpy(), g["obsB"][:, t])
        exp_state = np.where(d[:, None], g["reset_state"][:, t], g["state"][:, t])
        assert np.array_equal(_state_matrix(env), exp_state), (name, t)
        exp_oA = np.where(d[:, None], g["reset_obs"][:, t, 0], g["obsA"][:, t])
        exp_oB = np.where(d[:, None], g["reset_obs"][:, t, 1], g["obsB"][:, t])
        assert np.array_equal(oA.cpu().numpy(), exp_oA) and np.array_equal(oB.cpu().numpy(), exp_oB)


AT_SCALE_KW = {
    "cfg": dict(paddle_speed=0.03, max_score=3, magnus_factor=0.025, restitution=1, friction=0.6,
                ball_speed_range=[0.03, 0.05], spin_range=[-5, 5], speed_scale_every=1, speed_increment=0.1),
    # mass != 1 and an odd radius: the device divides by mass and inertia through their reciprocals
    "mass": dict(paddle_speed=0.041, max_score=5, magnus_factor=0.031, restitution=0.83, friction=0.35,
                 ball_mass=1.7, world_ball_radius=0.0123, ball_speed_range=[0.03, 0.05], spin_range=[-5, 5],
                 speed_scale_every=3, speed_increment=0.07),
}


@pytest.mark.parametrize("n,cfg", [(1, "cfg"), (255, "cfg"), (65536, "cfg"), (65536, "mass")])
def test_env_step_matches_oracle_at_scale(orc, n, cfg):
    """n arenas from random mid-game states (including y beyond the lines, paddles at the walls),
    random actions, 40 ticks without reset: bit-exact with the C oracle."""
    from pongmi.env import PongEnv2PBatch

    kw = AT_SCALE_KW[cfg]
    P = orc.make_params(orc.env_params_from_kwargs(**kw))
    rng = np.random.RandomState(n)
    st = dict(x=rng.uniform(-0.02, 1.02, n), y=rng.uniform(-0.05, 1.05, n), vx=rng.uniform(-0.08, 0.08, n),
              vy=rng.uniform(-0.08, 0.08, n), spin=rng.uniform(-6, 6, n), top=rng.choice([0.0, 0.5, 1.0, 0.31], n),
              bot=rng.uniform(0, 1, n), scoreA=rng.randint(0, 3, n), scoreB=rng.randint(0, 3, n),
              bounces=rng.randint(0, 9, n), serves=np.zeros(n))
    env = PongEnv2PBatch(n, **kw)
    env.set_state(st)
    arr = orc.arenas_from_soa(st)
    for t in range(40):
        aA = rng.randint(0, 3, n).astype(np.int8)
        aB = rng.randint(0, 3, n).astype(np.int8)
        (oA, oB), (rA, rB), done, _ = env.step(torch.from_numpy(aA), torch.from_numpy(aB))
        eA, eB, rew, ed = orc.step_arenas(P, arr, aA, aB)
        assert np.array_equal(done.cpu().numpy(), ed)
        assert np.array_equal(rA.cpu().numpy(), rew[:, 0]) and np.array_equal(rB.cpu().numpy(), rew[:, 1])
        assert np.array_equal(oA.cpu().numpy(), eA) and np.array_equal(oB.cpu().numpy(), eB)
    got = env.get_state()
    for k in STATE_ORDER:
        assert np.array_equal(got[k], arr[k]), k


def test_autoreset_done_rows_only():
    """autoreset='done' (ABI mode 2) against autoreset=True on the same Philox serves: identical
    state, obs, rewards and done every step; term rows written exactly for done arenas, with the
    full-mode values; every other row keeps its previous contents."""
    from pongmi.env import PongEnv2PBatch

    n = 65536
    full = PongEnv2PBatch(n, seed=5, autoreset=True)
    part = PongEnv2PBatch(n, seed=5, autoreset="done")
    full.reset()
    part.reset()
    g = torch.Generator(device="cuda").manual_seed(3)
    fill = torch.full((n, 7), -7.0, device="cuda")
    part.term_obsA.copy_(fill)
    part.term_obsB.copy_(fill)
    seen = 0
    for t in range(120):
        aA = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=g)
        aB = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=g)
        prevA, prevB = part.term_obsA.clone(), part.term_obsB.clone()
        (fA, fB), (frA, frB), fd, finfo = full.step(aA, aB)
        (pA, pB), (prA, prB), pd, pinfo = part.step(aA, aB)
        assert torch.equal(fA, pA) and torch.equal(fB, pB) and torch.equal(fd, pd)
        assert torch.equal(frA, prA) and torch.equal(frB, prB)
        d = pd.bool()
        seen += int(d.sum())
        for side, prev in (("term_obsA", prevA), ("term_obsB", prevB)):
            exp = torch.where(d[:, None], finfo[side], prev)
            assert torch.equal(pinfo[side], exp), (t, side)
    assert np.array_equal(_state_matrix(full), _state_matrix(part))
    assert seen > 1000


def test_autoreset_serves_match_philox_restatement(orc):
    """Production autoreset serves of pm_env_step (the branch-free reset): every arena that
    finishes in step t is served Philox(seed; i, TAG_SERVE_STEP, t) as the oracle restates it
    (cos/sin within 1 ulp of libm), serves[] is left alone (ABI 15: the step-keyed draw reads no
    counter), and every other arena ticks as the C oracle does."""
    from pongmi.env import PongEnv2PBatch

    n = 65536
    kw = dict(ball_speed_range=[0.03, 0.05], spin_range=[-5, 5], max_score=1)
    p = orc.env_params_from_kwargs(**kw)
    P = orc.make_params(p)
    env = PongEnv2PBatch(n, seed=77, autoreset=True, **kw)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(9)
    served = 0
    for t in range(60):
        before = env.get_state()
        aA = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=g)
        aB = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=g)
        _, _, done, _ = env.step(aA, aB)
        d = done.cpu().numpy().astype(bool)
        st = env.get_state()
        arr = orc.arenas_from_soa(before)
        _, _, _, ed = orc.step_arenas(P, arr, aA.cpu().numpy(), aB.cpu().numpy())
        assert np.array_equal(d, ed.astype(bool))
        for k in STATE_ORDER:
            assert np.array_equal(st[k][~d], arr[k][~d]), (t, k)
        idx = np.nonzero(d)[0]
        assert np.array_equal(st["serves"], before["serves"])
        assert env.counter == t + 1
        vx, vy, sp = orc.philox_serve(p, idx, None, 77, step=t)
        assert np.array_equal(st["vx"][idx], vx)
        assert np.array_equal(st["vy"][idx], vy)
        assert np.array_equal(st["spin"][idx], sp)
        for k, v in (("x", 0.5), ("y", 0.5), ("top", 0.5), ("bot", 0.5), ("scoreA", 0), ("scoreB", 0), ("bounces", 0)):
            assert np.all(st[k][idx] == v), (t, k)
        served += len(idx)
    assert served > 5000


def test_env_empty_and_bad_arguments():
    from pongmi import _lib
    from pongmi.env import PongEnv2PBatch, env_params

    env = PongEnv2PBatch(0)
    env.reset()
    env.step(np.zeros(0, np.int8), np.zeros(0, np.int8))
    with pytest.raises(ZeroDivisionError):
        env_params(speed_scale_every=0)
    with pytest.raises(TypeError):
        env_params(bogus=1)
    with pytest.raises(ValueError):
        PongEnv2PBatch(4).step(np.zeros(3), np.zeros(4))
    with pytest.raises(ValueError):
        PongEnv2PBatch(4, autoreset="sometimes")
    with pytest.raises(_lib.PongmiError):
        _lib.check(_lib.load().pm_env_step(None, None, None, None, None, None, None, None, None, None, None, 0, None,
                                           0, 0, 0, None, 4, None))
    with pytest.raises(_lib.PongmiError):
        _lib.check(_lib.load().pm_env_step(None, None, None, None, None, None, None, None, None, None, None, 0, None,
                                           0, 0, 0, None, -1, None))


def test_production_serves_match_philox_restatement(orc):
    """Philox serves: distribution of speed/angle/spin as reset() draws them, and each value equal
    to the oracle's Philox restatement (cos/sin within 1 ulp of libm)."""
    from pongmi.env import PongEnv2PBatch

    n = 200000
    kw = dict(ball_speed_range=[0.03, 0.05], spin_range=[-5, 5])
    env = PongEnv2PBatch(n, seed=1234, **kw)
    env.reset()
    st = env.get_state()
    p = orc.env_params_from_kwargs(**kw)
    vx, vy, sp = orc.philox_serve(p, np.arange(n), np.zeros(n, np.int64), 1234)
    assert np.array_equal(st["vx"], vx)
    assert np.array_equal(st["vy"], vy)
    assert np.array_equal(st["spin"], sp)
    speed = np.hypot(st["vx"], st["vy"])
    ang = np.degrees(np.arctan2(st["vy"], st["vx"]))
    assert speed.min() >= 0.03 - 1e-12 and speed.max() <= 0.05 + 1e-12
    assert np.all(((ang >= -60 - 1e-9) & (ang <= -30 + 1e-9)) | ((ang >= 30 - 1e-9) & (ang <= 60 + 1e-9)))
    assert abs(np.mean(ang > 0) - 0.5) < 0.01 and abs(np.mean(sp)) < 0.05
    assert np.all(st["serves"] == 1) and np.all(st["x"] == 0.5) and np.all(st["top"] == 0.5)


def test_collide_kat_bit_exact(golden):
    from pongmi import _lib

    g = golden("collide_kat")
    inp = g["inputs"]
    inertia = np.array([(2 / 5) * r[6] * r[7] ** 2 for r in inp])  # CPython's I (physics.py:9)
    d_in = torch.from_numpy(np.ascontiguousarray(inp)).cuda()
    d_I = torch.from_numpy(inertia).cuda()
    out = torch.empty((len(inp), 3), dtype=torch.float64, device="cuda")
    _lib.check(_lib.load().pm_collide(d_in.data_ptr(), d_I.data_ptr(), out.data_ptr(), len(inp), _lib.stream_ptr()))
    got = out.cpu().numpy()
    assert np.array_equal(got, g["outputs"])
    assert np.array_equal(np.signbit(got), np.signbit(g["outputs"]))


def test_scalar_dropin_matches_reference_trajectories_bit_exact(golden):
    """The scalar drop-in (envs/my_pong_env_2p.py PongEnv2P: one pm_env_reset1 / pm_env_step1 launch
    per call, results read from host-mapped memory) replays the reference's own runs exactly as
    make_golden.py recorded them: random.seed(seed_i), construct (one reset), then the recorded
    actions with reset() on done — every observation, reward, done flag and fp64 state word."""
    import random
    from envs.my_pong_env_2p import PongEnv2P

    g = golden("env_cfg")
    kw, _ = _kwargs_from_golden(g)
    n, T = g["actA"].shape
    for i in range(min(n, 6)):
        random.seed(int(g["seeds"][i]))
        env = PongEnv2P(**kw)
        assert np.array_equal(_state_matrix(env._env)[0], g["init"][i])
        oA, oB = env._get_obs()
        assert np.array_equal(oA, g["init_obs"][i, 0]) and np.array_equal(oB, g["init_obs"][i, 1])
        for t in range(T):
            (nA, nB), (rA, rB), d, info = env.step(int(g["actA"][i, t]), int(g["actB"][i, t]))
            assert info == {} and isinstance(d, bool)
            assert np.array_equal(nA, g["obsA"][i, t]) and np.array_equal(nB, g["obsB"][i, t]), (i, t)
            assert (rA, rB) == tuple(g["rew"][i, t].tolist()) and d == bool(g["done"][i, t]), (i, t)
            assert np.array_equal(_state_matrix(env._env)[0], g["state"][i, t]), (i, t)
            if d:
                oA, oB = env.reset()
                assert np.array_equal(oA, g["reset_obs"][i, t, 0]) and np.array_equal(oB, g["reset_obs"][i, t, 1])
                assert np.array_equal(_state_matrix(env._env)[0], g["reset_state"][i, t]), (i, t)
    with pytest.raises(ValueError):
        env.step(3, 0)


def test_scalar_collide_dropin_kat_bit_exact(golden):
    """envs/physics.py collide_sphere_with_moving_plane (pm_collide1, one launch per call) on the
    reference's collision known-answer table: bit-exact, signed zeros included."""
    from envs.physics import collide_sphere_with_moving_plane

    g = golden("collide_kat")
    got = np.array([collide_sphere_with_moving_plane(*[float(v) for v in r]) for r in g["inputs"]], np.float64)
    assert np.array_equal(got, g["outputs"])
    assert np.array_equal(np.signbit(got), np.signbit(g["outputs"]))
