"""The fused self-play learner (pm_selfplay_*) against the oracle, step by step:
rollout (acting + env tick + replay push + bookkeeping), learn (PER sample + double-DQN grads +
priority update) and apply (Adam + target sync + epsilon decay + counters)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ENV_KW = dict(paddle_speed=0.03, max_score=3, magnus_factor=0.025, restitution=1, friction=0.6,
              ball_speed_range=[0.03, 0.05], spin_range=[-5, 5], speed_scale_every=1, speed_increment=0.1)


def _sd(g, who):
    return {k[len(who) + 1:]: torch.from_numpy(v) for k, v in g.items() if k.startswith(who + ".") and "q_" not in k}


def _random_qnet_sd(seed):
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pingpong-selfplay-ai_amd"))
    from models.qnet import QNet
    torch.manual_seed(seed)
    return {k: v.clone() for k, v in QNet(7, 3).state_dict().items()}


def _learner(golden, n=2048, batch=256, cap=8192, n_pool=2, **kw):
    from pongmi.selfplay import SelfPlayLearner
    g = golden("qnet")
    pool = [_random_qnet_sd(100 + k) for k in range(n_pool)]
    return SelfPlayLearner(ENV_KW, n, _sd(g, "modelB"), _sd(g, "modelA"), pool, batch=batch, memory_size=cap,
                           epsilon=kw.pop("epsilon", 0.3), target_update_interval=kw.pop("target_update_interval", 3),
                           seed=kw.pop("seed", 5), **kw)


def _snap(L):
    torch.cuda.synchronize()
    return dict(f64=L.f64.cpu().numpy().copy(), i32=L.i32.cpu().numpy().copy(), opp=L.opp.cpu().numpy().copy(),
                er=L.ep_reward.cpu().numpy().copy(), ctrl=L.counters(), aA=L.aA.cpu().numpy().copy(),
                aB=L.aB.cpu().numpy().copy(), trans=L.trans.cpu().numpy().copy(),
                prios=L.prios.cpu().numpy().copy(), paramsB=L.paramsB.cpu().numpy().copy(),
                paramsT=L.paramsT.cpu().numpy().copy(), w_B=L.w_B.cpu().numpy().copy(),
                w_opp=L.w_opp.cpu().numpy().copy(), m=L.adam_m.cpu().numpy().copy(), v=L.adam_v.cpu().numpy().copy())


def _eff_from_w(w):
    """Effective-weight block (PM_QNET_NW) -> oracle eff dict."""
    w = w.astype(np.float64)
    return {"W1": w[:448].reshape(64, 7), "b1": w[448:512], "W2": w[512:4608].reshape(64, 64), "b2": w[4608:4672],
            "fc_V.W": w[4672:4736].reshape(1, 64), "fc_A.W": w[4736:4928].reshape(3, 64),
            "fc_V.b": w[4928:4929], "fc_A.b": w[4929:4932]}


def _check_rollout(orc, L, pre, post):
    """Replay one rollout on the oracle from the `pre` snapshot and compare with `post`."""
    n = L.n
    sp = L.sp
    pv = orc.env_params_from_kwargs(**ENV_KW)
    P = orc.make_params(pv)
    names = ("x", "y", "vx", "vy", "spin", "top", "bot")
    arr = np.zeros(n, orc.ARENA_DTYPE)
    for j, k in enumerate(names):
        arr[k] = pre["f64"][j]
    for j, k in enumerate(("scoreA", "scoreB", "bounces")):
        arr[k] = pre["i32"][j]
    oA, oB = orc.obs_of_arenas(arr)
    c = pre["ctrl"]
    step = c["step"]
    # both players' Q in the float32 restatement of the device's evaluation order (bitwise equal to
    # the matrix-core tile), so every arena's greedy action is checked, near-ties included
    qa = np.zeros((n, 3), np.float32)
    for k in range(L.n_pool + 1):
        sel = pre["opp"] == k
        qa[sel] = orc.qnet_forward_f32(pre["w_opp"][k], oA[sel])
    qb = orc.qnet_forward_f32(pre["w_B"], oB)
    r = orc.philox64(np.arange(n), orc.TAG_ACT, np.full(n, step, np.uint64), sp.seed_env)
    explore = orc.u53(r[0], r[1]) < c["epsilon"]
    aA = np.argmax(qa, 1)
    aB = np.where(explore, orc.below(r[2], 3), np.argmax(qb, 1))
    nA, nB, rew, done = orc.step_arenas(P, arr, aA.astype(np.int8), aB.astype(np.int8))
    d = done.astype(bool)
    # replay rows pushed at (pos + i) % cap
    slots = (c["pos"] + np.arange(n)) % L.cap
    rows = post["trans"][slots]
    assert np.array_equal(post["aA"], aA) and np.array_equal(post["aB"], aB)  # every arena
    assert np.array_equal(rows[:, 0:7], oB)
    assert np.array_equal(rows[:, 7], rew[:, 1])
    assert np.array_equal(rows[:, 8:15], nB)
    bits = rows[:, 15].view(np.int32)
    assert np.array_equal(bits & 0xFF, aB) and np.array_equal((bits >> 8) & 1, done)
    maxp = 1.0 if c["size"] == 0 else c["max_prio"]
    assert np.all(post["prios"][slots] == np.float32(maxp))
    # bookkeeping and serves
    er = pre["er"] + rew[:, 1]
    ns = pre["i32"][3]
    q = orc.philox(np.arange(n), orc.TAG_OPP, ns, 0, sp.seed_env)
    use_pool = (L.n_pool > 0) & (orc.u53(q[0], q[1]) < sp.pool_ratio)
    newopp = np.where(use_pool, 1 + orc.below(q[2], max(L.n_pool, 1)), 0)
    vx, vy, spn = orc.philox_serve(pv, np.arange(n), ns, sp.seed_env)
    m = d
    assert np.array_equal(post["opp"][m], newopp[m]) and np.array_equal(post["opp"][~d], pre["opp"][~d])
    assert np.all(post["er"][m] == 0) and np.array_equal(post["er"][~d], er[~d])
    assert np.all(post["i32"][3][m] == ns[m] + 1)
    assert np.array_equal(post["f64"][2][m], vx[m])
    assert np.array_equal(post["f64"][3][m], vy[m])
    assert np.array_equal(post["f64"][4][m], spn[m]) and np.all(post["f64"][0][m] == 0.5)
    keep = ~d
    for j, k in enumerate(names):
        assert np.array_equal(post["f64"][j][keep], arr[k][keep]), k
    for j, k in enumerate(("scoreA", "scoreB", "bounces")):
        assert np.array_equal(post["i32"][j][keep], arr[k][keep]), k
    win = er > 0
    return dict(fin=int(d.sum()), finA=int((d & (pre["opp"] == 0)).sum()), winA=int((d & (pre["opp"] == 0) & win).sum()),
                finP=int((d & (pre["opp"] != 0)).sum()), winP=int((d & (pre["opp"] != 0) & win).sum()),
                rsum=int(er[d].sum()))


def _check_per(orc, prios, size, cap, beta, u, idx, isw):
    """The update's PER draw, every one of its `batch` samples: indices and IS weights equal the
    restatement of the device's sum-tree descent (oracle.per_sample_tree, its own fp64 summation
    order) exactly; against np.random.choice's float32-normalised CDF (oracle.per_sample, the
    reference's algorithm) the indices are equal on every draw outside the CDF-boundary rounding band
    (oracle.per_boundary_band), and the band's count is printed (expected 0 or a few at 1e5+
    entries). Returns the normalised weights."""
    tidx, tw = orc.per_sample_tree(prios, size, cap, beta, u)
    assert np.array_equal(idx, tidx), f"{(idx != tidx).sum()} PER indices differ from the tree restatement"
    np.testing.assert_allclose(isw, tw, rtol=1.2e-7)  # one float32 ulp: the fp64 pow's last bit
    ref_idx, ref_w = orc.per_sample(prios, size, len(u), beta, u)
    band = orc.per_boundary_band(prios, size, u)
    assert np.array_equal(idx[~band], ref_idx[~band])
    print(f"PER: size {size}, {int(band.sum())} of {len(u)} draws in the CDF rounding band, "
          f"{int((idx != ref_idx).sum())} differ from np.random.choice's there")
    w = isw / isw.max()
    np.testing.assert_allclose(w, ref_w, rtol=3e-5)  # every draw
    return w


def test_rollout_matches_oracle(orc, golden):
    L = _learner(golden, n=4096, cap=16384, epsilon=0.3)
    for _ in range(12):
        pre = _snap(L)
        L.rollout()
        post = _snap(L)
        cnt = _check_rollout(orc, L, pre, post)
        L.learn()
        after = L.counters()
        assert after["ep_step"] == cnt["fin"]
        assert after["episodes"] - pre["ctrl"]["episodes"] == cnt["fin"]
        assert after["ep_A"] - pre["ctrl"]["ep_A"] == cnt["finA"] and after["win_A"] - pre["ctrl"]["win_A"] == cnt["winA"]
        assert after["ep_P"] - pre["ctrl"]["ep_P"] == cnt["finP"] and after["win_P"] - pre["ctrl"]["win_P"] == cnt["winP"]
        L.apply()


def test_learn_and_apply_match_oracle(orc, golden):
    """Each update: PER indices from the Philox uniforms on the pre-update priorities, loss and all
    520 head gradients from the oracle's double-DQN restatement with the update's own noise, the
    priority scatter, then Adam and the target sync."""
    L = _learner(golden, n=1024, batch=256, cap=4096, epsilon=0.5, target_update_interval=3, fuse_apply=False)
    sp = L.sp
    m_ref = np.zeros(520)
    v_ref = np.zeros(520)
    updates = 0
    for step in range(9):
        L.rollout()
        pre = _snap(L)
        L.learn()
        torch.cuda.synchronize()
        c = pre["ctrl"]
        size = min(c["size"] + L.n, L.cap)
        assert size >= L.batch
        frame = c["frame_idx"] + 1
        beta = min(1.0, 0.4 + frame * 0.6 / 100000)
        r = orc.philox64(np.arange(L.batch), orc.TAG_PER, np.full(L.batch, frame, np.uint64), sp.seed_env)
        u = orc.u53(r[0], r[1])
        idx = L.idx.cpu().numpy()
        w = _check_per(orc, pre["prios"], size, L.cap, beta, u, idx, L.isw.cpu().numpy())
        rows = pre["trans"][idx]
        s, ns = rows[:, 0:7], rows[:, 8:15]
        rwd = rows[:, 7]
        bits = rows[:, 15].view(np.int32)
        a, dn = bits & 0xFF, ((bits >> 8) & 1).astype(bool)
        from pongmi.qnet import unpack_state_dict
        sdB = {k: v.numpy() for k, v in unpack_state_dict(L.paramsB).items()}  # eps = the update's noise
        fVi, fVo, fAi, fAo = orc.philox_noise(sp.seed_net, orc.TAG_NOISE_TRAIN, c["train_steps"] + 1)
        assert np.array_equal(sdB["fc_A.weight_epsilon"], np.outer(fAo, fAi))
        heads = orc.pack_heads({k: v for k, v in sdB.items()})
        theads = orc.pack_heads({k: v.numpy() for k, v in unpack_state_dict(L.paramsT).items()})
        res = orc.dqn_loss_grads(sdB, heads, theads, sdB, s, a, rwd, ns, dn, w, 0.99)
        grad = L.grad.cpu().numpy()
        np.testing.assert_allclose(grad[:520], res["grads"], rtol=2e-4, atol=2e-6)
        assert grad[521] == 1.0
        np.testing.assert_allclose(L.counters()["last_loss"], res["loss"], rtol=1e-4)
        pr = L.prios.cpu().numpy()
        exp_pr = pre["prios"].copy()
        orc.per_update(exp_pr, idx, res["errors"])
        np.testing.assert_allclose(pr, exp_pr, rtol=2e-5, atol=3e-5)  # |q-t| carries fp32 error
        assert np.isclose(L.counters()["max_prio"], max(c["max_prio"], exp_pr[idx].max()), rtol=2e-5, atol=3e-5)
        L.apply()
        updates += 1
        p_ref, m_ref, v_ref = orc.adam_step(heads, grad[:520].astype(np.float64), m_ref, v_ref, updates, 2.5e-4)
        np.testing.assert_allclose(L.paramsB.cpu().numpy()[4672:5192], p_ref, rtol=1e-5, atol=1e-7)
        after = L.counters()
        assert after["train_steps"] == updates and after["frame_idx"] == updates
        if updates % 3 == 0:
            assert np.array_equal(L.paramsT.cpu().numpy()[:5192], L.paramsB.cpu().numpy()[:5192])
        else:
            assert np.array_equal(L.paramsT.cpu().numpy(), pre["paramsT"])
        D = grad[520]
        exp_eps = max(0.02, c["epsilon"] * 0.995 ** D)
        assert np.isclose(after["epsilon"], exp_eps, rtol=1e-12)
        assert after["step"] == c["step"] + 1 and after["pos"] == (c["pos"] + L.n) % L.cap
        assert after["size"] == size


def test_production_size_step_matches_oracle(orc, golden):
    """configs[2] at its full size (the bench's workload: 65 536 arenas, replay cap 1e6, batch 256,
    pool 8): the rollout of every arena and the update's PER draw, loss, head gradients and priority
    scatter against the oracle, over vector steps with the replay still filling."""
    L = _learner(golden, n=65536, batch=256, cap=1_000_000, n_pool=8, epsilon=0.3, fuse_apply=False)
    sp = L.sp
    for step in range(3):
        pre = _snap(L)
        L.rollout()
        post = _snap(L)
        _check_rollout(orc, L, pre, post)
        L.learn()
        torch.cuda.synchronize()
        c = pre["ctrl"]
        size = min(c["size"] + L.n, L.cap)
        frame = c["frame_idx"] + 1
        beta = min(1.0, 0.4 + frame * 0.6 / 100000)
        r = orc.philox64(np.arange(L.batch), orc.TAG_PER, np.full(L.batch, frame, np.uint64), sp.seed_env)
        idx = L.idx.cpu().numpy()
        w = _check_per(orc, post["prios"], size, L.cap, beta, orc.u53(r[0], r[1]), idx, L.isw.cpu().numpy())
        rows = post["trans"][idx]
        bits = rows[:, 15].view(np.int32)
        a, dn = bits & 0xFF, ((bits >> 8) & 1).astype(bool)
        from pongmi.qnet import unpack_state_dict
        sdB = {k: v.numpy() for k, v in unpack_state_dict(L.paramsB).items()}
        heads = orc.pack_heads(sdB)
        theads = orc.pack_heads({k: v.numpy() for k, v in unpack_state_dict(L.paramsT).items()})
        res = orc.dqn_loss_grads(sdB, heads, theads, sdB, rows[:, 0:7], a, rows[:, 7], rows[:, 8:15], dn, w, 0.99)
        grad = L.grad.cpu().numpy()
        np.testing.assert_allclose(grad[:520], res["grads"], rtol=2e-4, atol=2e-6)
        np.testing.assert_allclose(L.counters()["last_loss"], res["loss"], rtol=1e-4)
        exp_pr = post["prios"].copy()
        orc.per_update(exp_pr, idx, res["errors"])
        np.testing.assert_allclose(L.prios.cpu().numpy(), exp_pr, rtol=2e-5, atol=3e-5)
        L.apply()
    assert L.counters()["train_steps"] == 3 and L.counters()["size"] == 3 * 65536


def test_no_update_before_batch_is_full(golden):
    """train_step returns while len(memory) < batch_size (:134): no Adam, counters still advance."""
    L = _learner(golden, n=300, batch=256, cap=1000)
    p0 = L.paramsB.cpu().numpy()[4672:5192].copy()
    L.step()  # size 300 >= 256 already after the first push -> an update happens
    assert L.counters()["train_steps"] == 1
    L2 = _learner(golden, n=257, batch=256, cap=600, seed=9)
    L2.step()
    c = L2.counters()
    assert c["train_steps"] == 1 and c["size"] == 257
    assert not np.array_equal(L.paramsB.cpu().numpy()[4672:5192], p0)


def test_long_run_invariants(golden):
    L = _learner(golden, n=8192, batch=256, cap=65536, epsilon=1.0, target_update_interval=50)
    eps_trace = []
    for k in range(200):
        L.step()
        if k % 20 == 19:
            c = L.counters()
            eps_trace.append(c["epsilon"])
            assert np.isfinite(c["last_loss"])
    c = L.counters()
    assert c["step"] == 200 and c["train_steps"] == 200 and c["size"] == 65536
    assert c["episodes"] == c["ep_A"] + c["ep_P"] and c["episodes"] > 8192
    assert abs(c["ep_P"] / c["episodes"] - 0.33) < 0.03
    assert all(a >= b for a, b in zip(eps_trace, eps_trace[1:])) and eps_trace[-1] >= 0.02
    assert np.isfinite(L.paramsB.cpu().numpy()).all() and np.isfinite(L.prios.cpu().numpy()).all()
    st = L.i32.cpu().numpy()
    assert st[0].max() < 3 and st[1].max() < 3  # finished episodes were re-served


def test_fused_apply_is_bitwise_identical(golden):
    """Unsharded learn+apply fused into one kernel must equal the split path bit for bit."""
    A = _learner(golden, n=2048, batch=256, cap=8192, seed=3, fuse_apply=True)
    B = _learner(golden, n=2048, batch=256, cap=8192, seed=3, fuse_apply=False)
    for _ in range(15):
        A.step()
        B.rollout()
        B.learn()
        B.apply()
    torch.cuda.synchronize()
    for name in ("paramsB", "paramsT", "adam_m", "adam_v", "prios", "trans", "f64", "i32", "w_B", "learn_heads",
                 "per_work", "idx", "isw", "grad"):
        assert torch.equal(getattr(A, name), getattr(B, name)), name
    ca, cb = A.counters(), B.counters()
    assert ca == cb


def test_deterministic_rerun(golden):
    """Same seed, same everything: two learners stay bitwise identical (the only atomics — the LDS
    duplicate-index set of the priority scatter — have order-independent results)."""
    A = _learner(golden, n=4096, batch=256, cap=16384, seed=11)
    B = _learner(golden, n=4096, batch=256, cap=16384, seed=11)
    for _ in range(20):
        A.step()
        B.step()
    torch.cuda.synchronize()
    for name in ("paramsB", "prios", "trans", "f64", "opp", "per_work", "idx"):
        assert torch.equal(getattr(A, name), getattr(B, name)), name


def test_launch_timer_leaves_results_unchanged(golden):
    """pm_timer_arm: a timed launch (hipExtLaunchKernel with begin/end events) computes exactly what
    the plain one does, reports a positive duration, and a read without a timed launch is an error."""
    from pongmi import _lib
    A = _learner(golden, n=4096, batch=256, cap=16384, seed=11)
    B = _learner(golden, n=4096, batch=256, cap=16384, seed=11)
    durations = []
    for k in range(20):
        A.step()
        if k % 3 == 0:
            _lib.timer_arm(_lib.PM_TIMER_ACTENV)
            _lib.timer_arm(_lib.PM_TIMER_LEARN)
        B.step()
        if k % 3 == 0:
            durations += [_lib.timer_read(_lib.PM_TIMER_ACTENV), _lib.timer_read(_lib.PM_TIMER_LEARN)]
    torch.cuda.synchronize()
    for name in ("paramsB", "prios", "trans", "f64", "opp", "per_work", "idx"):
        assert torch.equal(getattr(A, name), getattr(B, name)), name
    assert all(0 < d < 0.1 for d in durations), durations
    with pytest.raises(_lib.PongmiError):
        _lib.timer_read(_lib.PM_TIMER_LEARN)
    with pytest.raises(_lib.PongmiError):
        _lib.timer_arm(_lib.PM_TIMER_N)


@pytest.mark.parametrize("n,cap", [(1000, 2500), (2048, 8192), (300, 1000), (4096, 4160),
                                   (65536, 1_000_000)])  # the last: the bench's configs[2] sizes
def test_sum_tree_incremental_equals_rebuild(golden, orc, n, cap):
    """The PER sum tree is maintained incrementally inside k_learn (scattered sub-blocks + the next
    push range, with the pending push substituted). After many steps — ring wrap-arounds at
    capacities that are not multiples of the 64/1024-entry nodes — it must equal a full rebuild
    (pm_selfplay_prepare) bit for bit, and the chunk sums must equal the oracle's (oracle.per_tree) exactly."""
    L = _learner(golden, n=n, batch=256, cap=cap, seed=4, epsilon=0.5)
    for k in range(3 * cap // n + 7):
        L.step()
    torch.cuda.synchronize()
    inc = L.per_work.clone()
    L.prepare()
    torch.cuda.synchronize()
    assert torch.equal(inc, L.per_work)
    nch = (cap + 1023) // 1024
    chunks = inc[:nch * 8].view(torch.float64).cpu().numpy()
    c = L.counters()
    pr = L.prios.cpu().numpy().astype(np.float32).copy()
    pos = c["pos"]
    slots = (pos + np.arange(n)) % cap  # the push the tree already accounts for
    pr[slots] = np.float32(c["max_prio"])
    ref, _, _ = orc.per_tree(pr, cap)  # the leaves prio ** 0.6 and the fp64 node sums in the device's order
    assert np.array_equal(chunks, ref)


def test_tree_refresh_timeout_is_repaired(golden, orc, monkeypatch):
    """a tree-refresh timeout (forced with the PONGMI_TR_FORCE_TIMEOUT hook: block 1's
    granule poll gives up at once) sets status bit 2 and leaves the sums stale; check_status raises;
    repair_tree rebuilds the tree (bit 2 -> bit 3), after which it equals the oracle's tree of the
    priorities exactly, check_status passes, and later incremental steps keep it equal to a rebuild."""
    from pongmi import _lib
    n, cap = 2048, 8192
    L = _learner(golden, n=n, batch=256, cap=cap, seed=4, epsilon=0.5)
    for _ in range(6):
        L.step()
    monkeypatch.setenv("PONGMI_TR_FORCE_TIMEOUT", "1")
    L.step()
    monkeypatch.delenv("PONGMI_TR_FORCE_TIMEOUT")
    c = L.counters()
    assert c["status"] & 4 and c["train_steps"] > 0, c
    with pytest.raises(_lib.PongmiError):
        L.check_status(c)
    stale = L.per_work.clone()

    def oracle_chunks():
        c = L.counters()
        pr = L.prios.cpu().numpy().astype(np.float32).copy()
        pr[(c["pos"] + np.arange(n)) % cap] = np.float32(c["max_prio"])  # the pending push
        return orc.per_tree(pr, cap)[0]

    nch = (cap + 1023) // 1024
    assert not np.array_equal(stale[:nch * 8].view(torch.float64).cpu().numpy(), oracle_chunks())  # stale indeed
    assert L.repair_tree(c) is True
    c = L.counters()
    assert c["status"] & 4 == 0 and c["status"] & 8
    L.check_status(c)
    assert L.repair_tree(c) is False
    assert np.array_equal(L.per_work[:nch * 8].view(torch.float64).cpu().numpy(), oracle_chunks())
    for _ in range(5):
        L.step()
    torch.cuda.synchronize()
    inc = L.per_work.clone()
    L.prepare()
    torch.cuda.synchronize()
    assert torch.equal(inc, L.per_work) and L.counters()["status"] == 8


def test_overlapped_step_is_bitwise_identical(golden):
    """pm_selfplay_step_overlap (the next step's side-A act in the learner's launch) must equal the
    plain step bit for bit, also across host changes of modelA (which invalidate the precomputed
    actions) and the bench's instrumented step shape (full act -> env -> learn_act -> apply)."""
    from pongmi import _lib
    A = _learner(golden, n=4096, batch=256, cap=16384, seed=21, n_pool=3)
    B = _learner(golden, n=4096, batch=256, cap=16384, seed=21, n_pool=3, overlap=False)
    for k in range(24):
        if k == 9:
            sd = _random_qnet_sd(77)
            A.set_modelA(sd)
            B.set_modelA(sd)
        if k % 5 == 3:  # instrumented shape
            A.act()
            A.env_step()
            A.learn(act_next=True)
            A.apply()
        else:
            A.step()
        B.step()
    B.act(_lib.PM_ACT_A)  # A already holds the next step's side-A actions
    torch.cuda.synchronize()
    for name in ("paramsB", "paramsT", "adam_m", "adam_v", "prios", "trans", "f64", "i32", "opp", "w_B",
                 "learn_heads", "per_work", "idx", "isw", "aA", "aB", "obsA", "obsB", "ep_reward"):
        assert torch.equal(getattr(A, name), getattr(B, name)), name
    assert A.counters() == B.counters()


@pytest.mark.parametrize("knobs", [{"PONGMI_PUSHG": "0"}, {"PONGMI_TR": "0"}, {"PONGMI_PUSH2": "0"},
                                   {"PONGMI_LATE_NOISE": "0"}, {"PONGMI_TR": "0", "PONGMI_PUSH2": "0"}])
def test_learner_variants_are_bitwise_identical(golden, monkeypatch, knobs):
    """k_learn's placement knobs (read per launch) move work between blocks and never change a
    result: the push rows as drained rows + flag instead of tagged granules (PUSHG=0, the
    k_learn<false> instantiation), the learner's own tree refresh instead of block 1's (TR=0), one wave
    per push-row tile (PUSH2=0), the apply's noise in phase 0 (LATE_NOISE=0). A push range of a
    quarter of the replay puts many sampled rows on the hand-off."""
    kw = dict(n=4096, batch=256, cap=16384, seed=31, n_pool=3)
    A = _learner(golden, **kw)
    B = _learner(golden, **kw)
    for _ in range(24):
        for k, v in knobs.items():
            monkeypatch.setenv(k, v)
        A.step()
        for k in knobs:
            monkeypatch.delenv(k)
        B.step()
    torch.cuda.synchronize()
    for name in ("paramsB", "paramsT", "adam_m", "adam_v", "prios", "trans", "f64", "i32", "opp", "w_B",
                 "learn_heads", "per_work", "idx", "isw", "aA", "aB", "obsA", "obsB", "ep_reward"):
        assert torch.equal(getattr(A, name), getattr(B, name)), name
    ca, cb = A.counters(), B.counters()
    assert ca == cb and ca["train_steps"] == 24 and ca["status"] == 0


def test_production_step_equals_plain_at_full_size(golden):
    """The bench's production step (overlapped, features ahead, fused apply) at configs[2]'s full
    size equals the plain three-kernel step bit for bit, across the replay ring's first wrap
    (1e6 / 65 536 = 15.3 vector steps) and a target sync."""
    kw = dict(n=65536, batch=256, cap=1_000_000, seed=23, n_pool=8, target_update_interval=10)
    A = _learner(golden, **kw)
    B = _learner(golden, overlap=False, features_ahead=False, fuse_apply=False, **kw)
    for _ in range(20):
        A.step()
        B.rollout()
        B.learn()
        B.apply()
    torch.cuda.synchronize()
    for name in ("paramsB", "paramsT", "adam_m", "adam_v", "prios", "trans", "f64", "i32", "opp", "w_B",
                 "learn_heads", "per_work", "idx", "isw", "aB", "obsA", "obsB", "ep_reward"):
        assert torch.equal(getattr(A, name), getattr(B, name)), name
    ca, cb = A.counters(), B.counters()
    assert ca == cb and ca["train_steps"] == 20 and ca["size"] == 1_000_000


def test_production_step_above_configs2_size(golden):
    """Above configs[2]'s arena count (262 144: the side-A act blocks alone fill the chip, so the
    feature blocks spread over the whole device) the production step still equals the
    plain step bit for bit, and the learner launch stays in the tens of µs (the old fallback put
    every feature tile on one block: ~8 000 tiles in series)."""
    from pongmi import _lib
    kw = dict(n=262144, batch=256, cap=1_000_000, seed=29, n_pool=8, target_update_interval=4)
    A = _learner(golden, **kw)
    B = _learner(golden, overlap=False, features_ahead=False, fuse_apply=False, **kw)
    for _ in range(8):
        A.step()
        B.rollout()
        B.learn()
        B.apply()
    torch.cuda.synchronize()
    for name in ("paramsB", "paramsT", "adam_m", "adam_v", "prios", "trans", "f64", "i32", "opp", "w_B",
                 "learn_heads", "per_work", "idx", "isw", "aB", "obsA", "obsB", "ep_reward"):
        assert torch.equal(getattr(A, name), getattr(B, name)), name
    assert A.counters() == B.counters()
    ts = []
    for _ in range(5):
        _lib.timer_arm(_lib.PM_TIMER_LEARN)
        A.step()
        ts.append(_lib.timer_read(_lib.PM_TIMER_LEARN))
    print(f"k_learn at 262144 arenas: {min(ts) * 1e6:.1f} us")
    assert min(ts) < 200e-6


def test_features_ahead_is_bitwise_identical(golden):
    """modelB's feature layers computed a launch ahead (the learner launch's feature blocks -> featB,
    k_actenv evaluates the heads only) equal k_actenv's full forward bit for bit, also across a
    reset_B (new feature weights: the precomputed features are invalidated and recomputed) and a
    ragged arena count (the last 32-row feature tile partial)."""
    for n in (4096, 3000):
        A = _learner(golden, n=n, batch=256, cap=16384, seed=23, n_pool=3)
        B = _learner(golden, n=n, batch=256, cap=16384, seed=23, n_pool=3, features_ahead=False)
        assert A.featB is not None and B.featB is None
        for k in range(20):
            if k == 11:
                sd = _random_qnet_sd(91)
                A.reset_B(sd, epsilon=0.2)
                B.reset_B(sd, epsilon=0.2)
            A.step()
            B.step()
        torch.cuda.synchronize()
        for name in ("paramsB", "paramsT", "adam_m", "adam_v", "prios", "trans", "f64", "i32", "opp", "w_B",
                     "learn_heads", "per_work", "idx", "isw", "aA", "aB", "obsA", "obsB", "ep_reward"):
            assert torch.equal(getattr(A, name), getattr(B, name)), (n, name)
        assert A.counters() == B.counters()
        assert A.counters()["train_steps"] > 0
        A.check_status()  # no push-row hand-off timed out


def test_sharded_world2_overlap_equals_plain(golden):
    """world = 2 on one device (rank-specific arenas / replay, one summed gradient): the overlapped
    sharded step (act B -> env -> learn with the next side-A act -> all-reduce -> k_adam) equals the
    plain sharded step (rollout -> learn -> all-reduce -> k_adam) bit for bit, and the two replicas'
    networks stay identical."""
    from pongmi import _lib

    def make(rank, overlap):
        return _learner(golden, n=2048, batch=256, cap=8192, seed=13, rank=rank, world=2, allreduce=lambda t: None,
                        overlap=overlap)

    ov = [make(0, True), make(1, True)]
    pl = [make(0, False), make(1, False)]
    for k in range(14):
        for L in ov:
            if not L._aA_ready:
                L.act(_lib.PM_ACT_A)
            if k % 2:
                L.act(_lib.PM_ACT_B)
                L.env_step()
            else:
                L.actenv()  # the fused launch: bit-identical to act B + env
            L.learn(act_next=True)
        for L in pl:
            L.rollout()
            L.learn()
        for pair in (ov, pl):
            g = pair[0].grad + pair[1].grad  # the all-reduce (SUM)
            for L in pair:
                L.grad.copy_(g)
                L.apply()
    torch.cuda.synchronize()
    for r in range(2):
        for name in ("paramsB", "paramsT", "adam_m", "adam_v", "prios", "trans", "f64", "i32", "opp", "w_B",
                     "learn_heads", "per_work", "idx", "isw", "aB", "obsA", "obsB", "ep_reward"):
            assert torch.equal(getattr(ov[r], name), getattr(pl[r], name)), (r, name)
        assert ov[r].counters() == pl[r].counters()
    for name in ("paramsB", "paramsT", "adam_m", "adam_v", "w_B", "learn_heads"):
        assert torch.equal(getattr(ov[0], name), getattr(ov[1], name)), name
    assert not torch.equal(ov[0].f64, ov[1].f64)  # rank-specific arenas
    assert ov[0].counters()["train_steps"] == 14


# ------------------------------------------------------------------------------ U > 1 updates per step
def _drive_split(L, U):
    """One vector step of U updates through the split entry points (rollout, learn_ex / apply_ex per
    update, resample for updates 1..U-1, commit)."""
    from pongmi import _lib
    L.rollout()
    for u in range(U):
        mode = _lib.PM_UPD_FIRST if u == 0 else 0
        if u:
            L.resample()
        L.learn_ex(mode)
        L.apply_ex(mode)
    L.commit()


def test_multi_update_step_matches_oracle(orc, golden):
    """U = 3 updates per vector step (replay ratio): update 0 samples with the push pending, updates
    1..2 resample the replay after it with their own frame (beta, Philox draw) and the update noise
    of their own train step; every update matches the oracle's double-DQN restatement and Adam; the
    commit sets max_prio to the array maximum exactly (U * batch >= n here, so scatters can lower it)
    and leaves the sum tree bit-identical to a full rebuild."""
    from pongmi import _lib
    from pongmi.qnet import unpack_state_dict
    U = 3
    L = _learner(golden, n=512, batch=256, cap=2048, epsilon=0.5, target_update_interval=4, fuse_apply=False,
                 overlap=False, updates_per_step=U)
    sp = L.sp
    m_ref, v_ref = np.zeros(520), np.zeros(520)
    updates = 0
    for step in range(6):
        c0 = L.counters()
        L.rollout()
        for u in range(U):
            mode = _lib.PM_UPD_FIRST if u == 0 else 0
            if u:
                L.resample()
            pre = _snap(L)
            L.learn_ex(mode)
            torch.cuda.synchronize()
            c = pre["ctrl"]
            assert c["step"] == c0["step"] and c["pos"] == c0["pos"]  # the step commits after its last update
            size = min(c["size"] + L.n, L.cap)
            frame = c["frame_idx"] + 1
            assert frame == updates + 1
            beta = min(1.0, 0.4 + frame * 0.6 / 100000)
            r = orc.philox64(np.arange(L.batch), orc.TAG_PER, np.full(L.batch, frame, np.uint64), sp.seed_env)
            # update 0's batch was drawn beside k_env with the push pending: the pushed priorities
            # are in pre["prios"] already, so every update samples from its snapshot
            idx = L.idx.cpu().numpy()
            w = _check_per(orc, pre["prios"], size, L.cap, beta, orc.u53(r[0], r[1]), idx, L.isw.cpu().numpy())
            rows = pre["trans"][idx]
            bits = rows[:, 15].view(np.int32)
            sdB = {k: v.numpy() for k, v in unpack_state_dict(L.paramsB).items()}
            fVi, fVo, fAi, fAo = orc.philox_noise(sp.seed_net, orc.TAG_NOISE_TRAIN, c["train_steps"] + 1)
            assert np.array_equal(sdB["fc_A.weight_epsilon"], np.outer(fAo, fAi))
            heads = orc.pack_heads(sdB)
            theads = orc.pack_heads({k: v.numpy() for k, v in unpack_state_dict(L.paramsT).items()})
            res = orc.dqn_loss_grads(sdB, heads, theads, sdB, rows[:, 0:7], bits & 0xFF, rows[:, 7], rows[:, 8:15],
                                     ((bits >> 8) & 1).astype(bool), w, 0.99)
            grad = L.grad.cpu().numpy()
            np.testing.assert_allclose(grad[:520], res["grads"], rtol=2e-4, atol=2e-6)
            exp_pr = pre["prios"].copy()
            orc.per_update(exp_pr, idx, res["errors"])
            np.testing.assert_allclose(L.prios.cpu().numpy(), exp_pr, rtol=2e-5, atol=3e-5)
            if u > 0:
                assert grad[520] == 0  # the step's episodes are counted by update 0 only
            L.apply_ex(mode)
            updates += 1
            p_ref, m_ref, v_ref = orc.adam_step(heads, grad[:520].astype(np.float64), m_ref, v_ref, updates, 2.5e-4)
            np.testing.assert_allclose(L.paramsB.cpu().numpy()[4672:5192], p_ref, rtol=1e-5, atol=1e-7)
            after = L.counters()
            assert after["train_steps"] == updates and after["frame_idx"] == updates
            if updates % 4 == 0:
                assert np.array_equal(L.paramsT.cpu().numpy()[:5192], L.paramsB.cpu().numpy()[:5192])
            if u == 0:
                assert np.isclose(after["epsilon"], max(0.02, c["epsilon"] * 0.995 ** grad[520]), rtol=1e-12)
            else:
                assert after["epsilon"] == c["epsilon"]
        L.commit()
        torch.cuda.synchronize()
        c = L.counters()
        pr = L.prios.cpu().numpy()
        assert c["max_prio"] == pr.max() and c["max_bits"] == 0
        assert c["step"] == c0["step"] + 1 and c["pos"] == (c0["pos"] + L.n) % L.cap
        assert c["size"] == min(c0["size"] + L.n, L.cap)
        inc = L.per_work.clone()
        L.prepare()
        torch.cuda.synchronize()
        assert torch.equal(inc, L.per_work), step


def test_multi_update_fused_equals_split(golden):
    """pm_selfplay_step_multi (overlapped, fused Adam) equals the split path bit for bit."""
    U = 4
    A = _learner(golden, n=1024, batch=256, cap=4096, seed=8, updates_per_step=U)
    B = _learner(golden, n=1024, batch=256, cap=4096, seed=8, updates_per_step=U, fuse_apply=False, overlap=False)
    for _ in range(9):
        A.step()
        _drive_split(B, U)
    torch.cuda.synchronize()
    for name in ("paramsB", "paramsT", "adam_m", "adam_v", "prios", "trans", "f64", "i32", "opp", "w_B",
                 "learn_heads", "per_work", "idx", "isw", "aB", "ep_reward"):
        assert torch.equal(getattr(A, name), getattr(B, name)), name
    assert A.counters() == B.counters()
    assert A.counters()["train_steps"] == 9 * U


def test_multi_update_sharded_replicas(golden):
    """world = 2 with U = 3: all-reduce after every update keeps the replicas identical."""
    from pongmi import _lib
    U = 3
    Ls = [_learner(golden, n=1024, batch=256, cap=4096, seed=13, rank=r, world=2, allreduce=lambda t: None,
                   updates_per_step=U, overlap=False) for r in range(2)]
    for _ in range(5):
        for L in Ls:
            L.rollout()
        for u in range(U):
            mode = _lib.PM_UPD_FIRST if u == 0 else 0
            for L in Ls:
                if u:
                    L.resample()
                L.learn_ex(mode)
            g = Ls[0].grad + Ls[1].grad
            for L in Ls:
                L.grad.copy_(g)
                L.apply_ex(mode)
        for L in Ls:
            L.commit()
    torch.cuda.synchronize()
    for name in ("paramsB", "paramsT", "adam_m", "adam_v", "w_B", "learn_heads"):
        assert torch.equal(getattr(Ls[0], name), getattr(Ls[1], name)), name
    c0, c1 = Ls[0].counters(), Ls[1].counters()
    assert c0["train_steps"] == c1["train_steps"] == 5 * U and c0["epsilon"] == c1["epsilon"]
    for L in Ls:
        assert L.counters()["max_prio"] == L.prios.cpu().numpy().max()


def _assert_same(A, B, names=("paramsB", "paramsT", "adam_m", "adam_v", "prios", "trans", "f64", "i32", "opp", "w_B",
                              "learn_heads", "per_work", "idx", "isw", "aB", "ep_reward", "grad")):
    torch.cuda.synchronize()
    for name in names:
        assert torch.equal(getattr(A, name), getattr(B, name)), name
    assert A.counters() == B.counters()


@pytest.mark.parametrize("n,cap,U,steps,sync", [(1024, 4096, 5, 12, 7), (65536, 1_000_000, 6, 18, 13)])
def test_learn_multi_equals_split(golden, n, cap, U, steps, sync):
    """Updates 1..U-1 of a vector step as ONE single-workgroup launch (k_learn_multi: features of s
    stored at push time, the tree's top level in LDS) equal the launch-per-update split path (resample +
    batch forward + learn_ex + apply_ex per update) bit for bit: parameters, Adam state, priorities,
    the whole sum tree, the acting / next-update weights, the last batch and its gradients, every
    counter; across the replay ring's wrap and target syncs inside a launch. configs[2]'s full size
    is the second case."""
    kw = dict(n=n, batch=256, cap=cap, seed=31, n_pool=3, updates_per_step=U, target_update_interval=sync)
    A = _learner(golden, **kw)
    B = _learner(golden, fuse_apply=False, overlap=False, **kw)
    assert A.frow is not None and B.frow is None and A.sp.frow_ready == 1
    for k in range(steps):
        A.step()
        _drive_split(B, U)
        if k % 5 == 4:
            _assert_same(A, B)
    _assert_same(A, B)
    assert A.counters()["train_steps"] == steps * U


def test_learn_multi_waits_for_stored_features(golden):
    """A push through k_env (rollout / env_step) stores no row features: the fused multi-update path
    stands down until those rows have left the ring (cap / n pushes), and a reset_B (empty replay)
    re-arms it at once; the results equal the split path throughout."""
    U, n, cap = 3, 1024, 4096
    kw = dict(n=n, batch=256, cap=cap, seed=37, n_pool=2, updates_per_step=U, target_update_interval=5)
    A = _learner(golden, **kw)
    B = _learner(golden, fuse_apply=False, overlap=False, **kw)
    ready = []
    for k in range(16):
        if k == 3:  # a plain push on A (the k_env path), the same step on B
            from pongmi import _lib
            A.act()
            A.env_step()
            for u in range(U):
                mode = _lib.PM_UPD_FIRST if u == 0 else 0
                if u:
                    A.resample()
                A.learn_ex(mode)
                A.apply_ex(mode)
            A.commit()
            _drive_split(B, U)
        elif k == 10:
            sd = _random_qnet_sd(93)
            A.reset_B(sd, epsilon=0.4)
            B.reset_B(sd, epsilon=0.4)
            ready.append(A.sp.frow_ready)
            A.step()
            _drive_split(B, U)
        else:
            A.step()
            _drive_split(B, U)
        ready.append(A.sp.frow_ready)
    _assert_same(A, B)
    assert ready[3] == 0 and ready[4] == 0 and 1 in ready[5:10] and ready[10] == 1
