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


# ---------------------------------------------------------------------------------------------------
# §8f3: the collecting rollout (pm_rollout_push) — the same launch with every transition pushed into
# the replay ring from registers. Checked bit for bit against the stepped composition above with the
# training loop's memory.push((oB, aB, rB, nB, done)) (scripts/train_iterative.py:242-243) applied
# on the host in arena order, ep_reward / win bookkeeping (:245-248), and the PER sum tree against a
# full rebuild from the priorities (pm_per_sample's build).


def _stepped_push(env, wA, paramsB, eps, seed_net, steps, ring, ep, prio, alpha):
    """`steps` stepped vector steps; pushes into the host ring dict (trans, prios, pos, cap)."""
    from pongmi import _lib
    from pongmi.qnet import act, fold
    n, cap = env.n, ring["cap"]
    tot = np.zeros(6, np.int64)
    for _ in range(steps):
        c = env.counter
        wB = fold(paramsB, _lib.PM_FOLD_TRAIN_FRESH, seed=seed_net, counter=c)
        aA, aB = act(wA.reshape(1, -1), None, wB, env.obsA, env.obsB, eps, seed=env.seed, counter=c)[:2]
        s = env.obsB.cpu().numpy().copy()
        _, (rA, rB), done, info = env.step(aA, aB)
        nB = info["term_obsB"].cpu().numpy()
        r = rB.cpu().numpy()
        d = done.cpu().numpy().astype(bool)
        a = aB.cpu().numpy().astype(np.int32)
        slot = (ring["pos"] + np.arange(n)) % cap
        ring["trans"][slot, 0:7] = s
        ring["trans"][slot, 7] = r
        ring["trans"][slot, 8:15] = nB
        ring["trans"][slot, 15] = (a | (d.astype(np.int32) << 8)).view(np.float32)
        ring["prios"][slot] = prio
        ring["pos"] = (ring["pos"] + n) % cap
        ep += r
        tot += np.array([d.sum(), (d & (r > 0)).sum(), (rA.cpu().numpy() > 0).sum(), (r > 0).sum(),
                         (d & (ep > 0)).sum(), int(ep[d].sum())])
        ep[d] = 0
    return tot


def _tree_equals_rebuild(replay):
    """The launch-maintained sum tree equals pm_per_sample's full rebuild from prios (size == cap)."""
    from pongmi import replay as rp
    assert replay.size == replay.cap
    rp.per_sample(replay.prios, replay.size, 8, 0.4, alpha=replay.alpha, seed=1)
    ref = rp._workspace(replay.cap, replay.prios.device).cpu()
    got = replay.work.cpu()
    nchunk, nsub = -(-replay.cap // 1024), -(-replay.cap // 64)
    o1 = rp._pad(nchunk)
    o2 = o1 + rp._pad(nsub)
    for lo, nbytes in ((0, 8 * nchunk), (o1, 8 * nsub), (o2, 4 * replay.cap)):  # chunk / sub sums, leaves
        assert torch.equal(got[lo:lo + nbytes], ref[lo:lo + nbytes]), lo


@pytest.mark.parametrize("n,cap,launches,eps", [(1000, 1000 * 50, (30, 40), 0.02), (333, 333 * 60, (35, 45), 1.0),
                                                (4096, 4096 * 24, (10, 14), 0.02)])
def test_collect_equals_stepped_push(n, cap, launches, eps):
    from pongmi.replay import DeviceReplay
    from pongmi.rollout import STATS_PUSH, SelfPlayRollout
    wA, paramsB = _models(n + 1)
    seed_env, seed_net = 0xC011 + n, 5 + n
    fused, ref = _env(n, seed_env), _env(n, seed_env)
    replay = DeviceReplay(cap, fused.device)
    roll = SelfPlayRollout(fused, wA, paramsB, epsilon=eps, seed_net=seed_net)
    ring = {"trans": np.zeros((cap, 16), np.float32), "prios": np.zeros(cap, np.float32), "pos": 0, "cap": cap}
    ep = np.zeros(n, np.float32)
    tot = np.zeros(6, np.int64)
    got = np.zeros(6, np.int64)
    for k, steps in enumerate(launches):
        if k == 1:  # priorities changed by a learner between launches: the next push stores their max
            g = torch.Generator().manual_seed(n)
            new = torch.rand(replay.size, generator=g) * 3 + 0.01
            replay.prios[:replay.size] = new.to(replay.prios.device)
            ring["prios"][:replay.size] = new.numpy()
            replay.refresh()
        prio = replay.push_prio()
        st = roll.run(steps, replay=replay)
        got += np.array([st[k2] for k2 in STATS_PUSH])
        tot += _stepped_push(ref, wA, paramsB, eps, seed_net, steps, ring, ep, np.float32(prio), replay.alpha)
    _same_env(fused, ref)
    assert got.tolist() == tot.tolist()
    assert replay.pos == ring["pos"] and replay.size == min(cap, sum(launches) * n)
    assert np.array_equal(replay.trans.cpu().numpy().view(np.int32), ring["trans"].view(np.int32))
    assert np.array_equal(replay.prios.cpu().numpy(), ring["prios"])
    assert np.array_equal(roll.ep_reward.cpu().numpy(), ep)
    assert got[0] > 0
    _tree_equals_rebuild(replay)


def test_collect_full_size_ring():
    """configs[2]'s arena count: 65 536 arenas, 15 vector steps in one launch fill a 983 040-row ring
    exactly; rows, tree and state against the stepped composition."""
    from pongmi.replay import DeviceReplay
    from pongmi.rollout import STATS_PUSH, SelfPlayRollout
    n, steps = 65536, 15
    cap = n * steps
    wA, paramsB = _models(11)
    fused, ref = _env(n, 0x5EED), _env(n, 0x5EED)
    replay = DeviceReplay(cap, fused.device)
    roll = SelfPlayRollout(fused, wA, paramsB, epsilon=0.02, seed_net=9)
    st = roll.run(steps, replay=replay)
    ring = {"trans": np.zeros((cap, 16), np.float32), "prios": np.zeros(cap, np.float32), "pos": 0, "cap": cap}
    ep = np.zeros(n, np.float32)
    tot = _stepped_push(ref, wA, paramsB, 0.02, 9, steps, ring, ep, np.float32(1.0), replay.alpha)
    _same_env(fused, ref)
    assert [st[k] for k in STATS_PUSH] == tot.tolist()
    assert np.array_equal(replay.trans.cpu().numpy().view(np.int32), ring["trans"].view(np.int32))
    assert np.array_equal(replay.prios.cpu().numpy(), ring["prios"])
    _tree_equals_rebuild(replay)


def test_collect_failure_paths():
    from pongmi import _lib
    from pongmi.replay import DeviceReplay
    from pongmi.rollout import SelfPlayRollout
    wA, paramsB = _models(2)
    env = _env(100, 3)
    roll = SelfPlayRollout(env, wA, paramsB)
    with pytest.raises(_lib.PongmiError):
        roll.run(3, replay=DeviceReplay(250, env.device))  # 300 pushes > cap: a slot written twice
    assert env.counter == 0
    r = DeviceReplay(300, env.device)
    assert roll.run(0, replay=r)["episodes"] == 0 and r.size == 0


def test_collect_without_tree_matches():
    """per_work = NULL (no PER leaves, no node rebuild): the same rows, priorities and state as with the
    tree; the host side's DeviceReplay always passes one, so this drives the C-ABI directly."""
    import ctypes
    from pongmi import _lib
    from pongmi._lib import ptr, stream_ptr
    from pongmi.env import ctypes_ref
    from pongmi.replay import DeviceReplay
    from pongmi.rollout import SelfPlayRollout
    n, steps = 500, 60
    wA, paramsB = _models(21)
    a, b = _env(n, 77), _env(n, 77)
    ra, rb = SelfPlayRollout(a, wA, paramsB, seed_net=4), SelfPlayRollout(b, wA, paramsB, seed_net=4)
    with_tree = DeviceReplay(n * steps, a.device)
    ra.run(steps, replay=with_tree)
    trans = torch.zeros((n * steps, 16), dtype=torch.float32, device=b.device)
    prios = torch.zeros(n * steps, dtype=torch.float32, device=b.device)
    rb.reserve(steps)
    stats = torch.zeros(6, dtype=torch.int64, device=b.device)
    rp = _lib.RollReplay(trans=ptr(trans), prios=ptr(prios), per_work=None, ep_reward=ptr(rb.ep_reward), pos=0,
                         cap=n * steps, prio=1.0, alpha=0.6)
    L = _lib.load()
    _lib.check(L.pm_rollout_push(ctypes_ref(b.params), ctypes_ref(b.state), ptr(rb.wA), ptr(rb.wB), ptr(rb.paramsB),
                                 rb.epsilon, b.seed, rb.seed_net, b.counter, steps, ptr(rb.heads), ptr(b.obsA),
                                 ptr(b.obsB), ctypes.byref(rp), ptr(stats), n, stream_ptr()), "pm_rollout_push")
    b.counter += steps
    _same_env(a, b)
    assert torch.equal(trans.view(torch.int32).cpu(), with_tree.trans.view(torch.int32).cpu())
    assert torch.equal(prios.cpu(), with_tree.prios.cpu())
    assert torch.equal(ra.ep_reward.cpu(), rb.ep_reward.cpu())
    assert int(stats[0]) > 0


# ---------------------------------------------------------------------------------------------------
# Both launches against the oracle directly (oracle.cpu_selfplay.PhiloxRollout: the rollout restated
# on the device's Philox streams — noise, epsilon draws, serves — with the QNet in the tile's float32
# order and the C oracle's tick), not only against the stepped HIP composition: rows (as int32),
# priorities, PER leaves and tree, the env state, observations, ep_reward and counters, bit for bit.
CFG = dict(paddle_width=0.2, paddle_speed=0.03, max_score=3, enable_spin=True, magnus_factor=0.025, restitution=1,
           friction=0.6, ball_mass=1.0, world_ball_radius=0.03, ball_speed_range=[0.03, 0.05], spin_range=[-5, 5],
           ball_angle_intervals=[[-60, -30], [30, 60]], speed_scale_every=1, speed_increment=0.1)  # config.yaml


def _nets(seed):
    from models.qnet import QNet
    from pongmi import _lib
    from pongmi.qnet import fold, pack_state_dict
    torch.manual_seed(seed)
    mA, mB = QNet(7, 3), QNet(7, 3)
    sdA = {k: v.numpy() for k, v in mA.state_dict().items()}
    sdB = {k: v.numpy() for k, v in mB.state_dict().items()}
    return sdA, sdB, fold(pack_state_dict(mA.state_dict()), _lib.PM_FOLD_TRAIN).reshape(-1), \
        pack_state_dict(mB.state_dict()).reshape(-1)


def _env_matches_oracle(env, o, orc):
    st = env.get_state()
    for k in ("x", "y", "vx", "vy", "spin", "top", "bot", "scoreA", "scoreB", "bounces"):
        assert np.array_equal(st[k], o.arr[k]), k
    oA, oB = orc.obs_of_arenas(o.arr)
    assert np.array_equal(env.obsA.cpu().numpy(), oA) and np.array_equal(env.obsB.cpu().numpy(), oB)
    assert env.counter == o.counter


@pytest.mark.parametrize("n,steps,eps", [(4096, 120, 0.02), (333, 80, 1.0), (1000, 100, 0.0)])
def test_rollout_matches_oracle(orc, n, steps, eps):
    """K9 (pm_rollout, configs[1]) against the oracle rollout: state, observations, counters."""
    from oracle.cpu_selfplay import PhiloxRollout
    from pongmi.env import PongEnv2PBatch
    from pongmi.rollout import STATS, SelfPlayRollout
    sdA, sdB, wA, paramsB = _nets(100 + n)
    seed_env, seed_net = 0x5EED + n, 31 + n
    env = PongEnv2PBatch(n, seed=seed_env, autoreset=True, **CFG)
    env.reset()
    o = PhiloxRollout(CFG, env.get_state(), sdA, sdB, eps, seed_env, seed_net, env.counter)
    assert np.array_equal(o.wA, wA.cpu().numpy()[:4932])  # modelA's fold (its frozen eps) restated
    st = SelfPlayRollout(env, wA, paramsB, epsilon=eps, seed_net=seed_net).run(steps)
    tot = o.run(steps)
    _env_matches_oracle(env, o, orc)
    assert [st[k] for k in STATS] == tot[:4].tolist()
    assert tot[0] > 0


@pytest.mark.parametrize("n,steps_per_launch,launches", [(4096, 12, 2), (65536, 15, 1)])
def test_collect_matches_oracle(orc, n, steps_per_launch, launches):
    """The collecting rollout (pm_rollout_push) against the oracle with memory.push: at 4 096 arenas
    over two launches, the ring wrapping inside the second and the priorities changed in between (the
    push then stores their max); at configs[2]'s 65 536 arenas, one 15-step launch filling a
    983 040-row ring exactly."""
    from oracle.cpu_selfplay import PhiloxRollout
    from pongmi.env import PongEnv2PBatch
    from pongmi.replay import DeviceReplay
    from pongmi.rollout import STATS_PUSH, SelfPlayRollout
    sdA, sdB, wA, paramsB = _nets(7 + n)
    seed_env, seed_net, eps = 0xC0DE + n, 11 + n, 0.02
    cap = n * steps_per_launch * launches - (n // 2 if launches > 1 else 0)  # wraps inside the last launch
    cap = max(cap, n * steps_per_launch)
    env = PongEnv2PBatch(n, seed=seed_env, autoreset=True, **CFG)
    env.reset()
    replay = DeviceReplay(cap, env.device)
    roll = SelfPlayRollout(env, wA, paramsB, epsilon=eps, seed_net=seed_net)
    ring = {"trans": np.zeros((cap, 16), np.float32), "prios": np.zeros(cap, np.float32), "pos": 0, "cap": cap}
    o = PhiloxRollout(CFG, env.get_state(), sdA, sdB, eps, seed_env, seed_net, env.counter, replay=ring)
    got = np.zeros(6, np.int64)
    for k in range(launches):
        if k == 1:  # a learner changed the priorities between the launches
            g = torch.Generator().manual_seed(n)
            new = torch.rand(replay.size, generator=g) * 3 + 0.01
            replay.prios[:replay.size] = new.to(replay.prios.device)
            ring["prios"][:replay.size] = new.numpy()
            replay.refresh()
        ring["prio"] = np.float32(ring["prios"].max() if k else 1.0)  # PrioritizedReplay.push's max (:57)
        assert np.float32(replay.push_prio()) == ring["prio"]
        st = roll.run(steps_per_launch, replay=replay)
        got += np.array([st[k2] for k2 in STATS_PUSH])
        o.run(steps_per_launch)
    _env_matches_oracle(env, o, orc)
    assert got.tolist() == o.stats.tolist()
    assert replay.pos == ring["pos"]
    assert np.array_equal(replay.trans.cpu().numpy().view(np.int32), ring["trans"].view(np.int32))
    assert np.array_equal(replay.prios.cpu().numpy(), ring["prios"])
    assert np.array_equal(roll.ep_reward.cpu().numpy(), o.ep_reward)
    # the PER leaves prio ** alpha and both node levels, restated (oracle.per_tree) from the oracle's prios
    from pongmi import replay as rp
    chunk, sub, leaf = orc.per_tree(ring["prios"], cap, replay.alpha)
    work = replay.work.cpu()
    nchunk, nsub = -(-cap // 1024), -(-cap // 64)
    o1 = rp._pad(nchunk)
    o2 = o1 + rp._pad(nsub)
    assert np.array_equal(work[:8 * nchunk].numpy().view(np.float64), chunk)
    assert np.array_equal(work[o1:o1 + 8 * nsub].numpy().view(np.float64), sub)
    assert np.array_equal(work[o2:o2 + 4 * cap].numpy().view(np.float32), leaf)
    assert got[0] > 0


@pytest.mark.parametrize("tiles", [0, 3, 7, 8, 19, 23, 35, 64])
def test_rollout_tile_variants_match_oracle(orc, monkeypatch, tiles):
    """Every rollout kernel against the oracle: PONGMI_ROLL16=0 runs the 32-arena-tile
    k_rollout (inference) and k_rollout_push (collecting, the default there); =3 runs the 16-arena-tile
    k_rollout16 (the inference default, head chains on the matrix cores) and k_rollout16_push (A/B
    only); =7 the same with k_rollout16's round-4 VALU head chains; =8 the 32-arena-tile kernels with
    the round-4 replicated tick (rollout_body; 0 runs the one-tick rollout_body1); 19 / 23 = 3 / 7 with
    k_rollout16's weights read from LDS every step (round 5) instead of held in registers; 35 = 3 with
    the MFMA heads' cross-lane moves through ds_bpermute instead of the permlane swaps; 64 = 0 with the
    one-tick bodies' serve draw as two Philox blocks in a row. The library reads the variable at each
    launch."""
    monkeypatch.setenv("PONGMI_ROLL16", str(tiles))
    test_rollout_matches_oracle(orc, 333, 40, 0.02)
    test_collect_matches_oracle(orc, 4096, 12, 2)
