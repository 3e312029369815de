"""The QNetRNN self-play loop (pm_rnn_selfplay_*, K7) — train_rnn_iterative.py:731-798 batched:

1. step by step against the oracle: each player's acting decision (select_action_for_model,
   :371-389) against the float64 QNetRNN restatement (oracle.rnn_forward) from the device's carried
   (h, c) (zeroed at episode start) — the new (h, c) and Q of every arena within the tolerances below,
   the epsilon branch's random action exact (Philox restated) with (h, c) still advanced, and every
   greedy action equal to the oracle's argmax wherever the oracle's top-2 Q gap is wider than twice
   the Q tolerance (the in-band count is reported); the env against the oracle env; the ring records
   push_step(obs_B, act_B, reward_B, next_obs_B, done) exactly, finished arenas redraw their
   opponent and re-serve (Philox), bookkeeping matches;
2. the sequence buffer: every stored episode is one contiguous trajectory of >= T steps ending in
   done, the latest memory_size are kept, sampled sequences are windows of stored episodes, the
   update runs exactly when len(memory) > batch * min_episodes_for_training_start, epsilon decays
   once per finished episode;
3. determinism, and two data-parallel ranks (gradient sum + contributing-rank count) stay identical.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ENV_KW = dict(paddle_width=0.2, paddle_speed=0.03, max_score=3, enable_spin=True, magnus_factor=0.025, restitution=1.0,
              friction=0.6, ball_mass=1.0, world_ball_radius=0.03, ball_speed_range=[0.03, 0.05],
              spin_range=[-5, 5], ball_angle_intervals=[[-60, -30], [30, 60]], speed_scale_every=5,
              speed_increment=0.2)  # config_rnn.yaml:6-28


def _rnn_sd(seed):
    from models.qnet_rnn import QNetRNN
    torch.manual_seed(seed)
    return {k: v.clone() for k, v in QNetRNN(7, 3).state_dict().items()}


def _golden_sd(g):
    return {k[7:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("params.")}


def _learner(golden, n=256, n_pool=2, **kw):
    from pongmi.rnn_selfplay import RNNSelfPlayLearner
    g = golden("rnn")
    pool = [_rnn_sd(200 + k) for k in range(n_pool)]
    return RNNSelfPlayLearner(ENV_KW, n, _golden_sd(g), _rnn_sd(7), pool, **kw)


def _snap(L):
    torch.cuda.synchronize()
    t = lambda x: x.detach().cpu().numpy().copy()  # noqa: E731
    return dict(f64=t(L.f64), i32=t(L.i32), opp=t(L.opp), er=t(L.ep_reward), el=t(L.ep_len), es=t(L.ep_steps),
                reset=t(L.reset),
                obsA=t(L.obsA), obsB=t(L.obsB), hA=L.hA.clone(), cA=L.cA.clone(), hB=L.hB.clone(), cB=L.cB.clone(),
                ctrl=L.counters())


# QNetRNN act on the device vs the float64 oracle: exact-f32 MFMA sums in another order plus the
# v_exp_f32 / v_rcp_f32 activations (a few ulp each): per element
# |device - oracle| <= ATOL + RTOL * |oracle| for the new h, c and for Q
RNN_ACT_ATOL, RNN_ACT_RTOL = 2e-5, 4e-5


def _check_rnn_act(who, a_dev, q_dev, h_dev, c_dev, q_or, h_or, c_or, eps, seed, ctr, arenas, orc):
    """One player's act of one vector step against the oracle. Returns (in-band arenas, explored)."""
    np.testing.assert_allclose(h_dev, h_or, rtol=RNN_ACT_RTOL, atol=RNN_ACT_ATOL, err_msg=f"{who}: h")
    np.testing.assert_allclose(c_dev, c_or, rtol=RNN_ACT_RTOL, atol=RNN_ACT_ATOL, err_msg=f"{who}: c")
    tol = RNN_ACT_ATOL + RNN_ACT_RTOL * np.abs(q_or)
    assert np.all(np.abs(q_dev - q_or) <= tol), f"{who}: Q off by {np.abs(q_dev - q_or).max():.3g}"
    want, explore = orc.rnn_act_decision(q_or, eps, seed, ctr, arenas)
    # the epsilon branch: randint(0, 2) from the restated Philox draw, exact
    assert np.array_equal(a_dev[explore], want[explore]), f"{who}: epsilon-branch actions"
    g = ~explore
    assert np.array_equal(a_dev[g], orc.argmax_first(q_dev)[g]), f"{who}: action != argmax of the launch's own Q"
    srt = np.sort(q_or, axis=1)
    band = srt[:, 2] - srt[:, 1] <= 2.0 * tol.max(axis=1)  # top-2 gap inside the proven error: either may win
    clear = g & ~band
    assert np.array_equal(a_dev[clear], want[clear]), \
        f"{who}: {np.count_nonzero(a_dev[clear] != want[clear])} greedy actions differ from the oracle's argmax"
    inb = g & band  # in the band: the device's pick is still one of the near-tied maxima
    qpick = q_or[np.arange(len(q_or)), a_dev.astype(np.int64)]
    assert np.all(qpick[inb] >= srt[inb, 2] - 2.0 * tol.max(axis=1)[inb]), f"{who}: in-band pick not a near-max"
    err = dict(q=float(np.max(np.abs(q_dev - q_or) / (RNN_ACT_ATOL + RNN_ACT_RTOL * np.abs(q_or)))),
               h=float(np.max(np.abs(h_dev - h_or) / (RNN_ACT_ATOL + RNN_ACT_RTOL * np.abs(h_or)))),
               c=float(np.max(np.abs(c_dev - c_or) / (RNN_ACT_ATOL + RNN_ACT_RTOL * np.abs(c_or)))),
               dq=float(np.max(np.abs(q_dev - q_or))), dh=float(np.max(np.abs(h_dev - h_or))),
               dc=float(np.max(np.abs(c_dev - c_or))), mismatch_in_band=int(np.count_nonzero(a_dev[inb] != want[inb])))
    return int(inb.sum()), int(explore.sum()), err


@pytest.mark.parametrize("n,max_steps,nsteps,eps", [(256, 1000, 60, 0.0), (256, 24, 60, 0.3), (32768, 1000, 40, 0.0),
                                                    (32768, 1000, 40, 0.3)])
def test_rnn_selfplay_steps_match_oracle(golden, orc, n, max_steps, nsteps, eps):
    """max_steps = 24 exercises the max_episode_steps cut (:751): the episode ends (new opponent,
    serve, zero (h, c), counters) but the trajectory goes on until a done. n = 32 768 is configs[4]'s
    full arena count; eps = 0.3 exercises modelB's epsilon branch (which still advances (h, c),
    :375-380) on ~30 % of the arenas, with epsilon decaying per finished episode."""
    from pongmi.rnn import unpack_state_dict
    # overlap=False: this test reads the opponents' (h, c) after every step, which the overlapped
    # step has already advanced for the next one (test_rnn_overlapped_step_is_bitwise_identical)
    pool_sds = [_rnn_sd(200 + k) for k in range(2)]
    from pongmi.rnn_selfplay import RNNSelfPlayLearner
    L = RNNSelfPlayLearner(ENV_KW, n, _golden_sd(golden("rnn")), _rnn_sd(7), pool_sds, epsilon=eps,
                           min_epsilon=0.0, pool_ratio=0.5, min_episodes_for_training_start=10 ** 6, memory_size=4096,
                           seed=3, max_episode_steps=max_steps, overlap=False, record_q=True)
    n, sp = L.n, L.sp
    # the opponents act in eval mode (mu only): modelA, then the pool nets (:609-621)
    effA = [orc.rnn_effective({k: v.numpy() for k, v in sd.items()}, False) for sd in [_rnn_sd(7)] + pool_sds]
    arenas = np.arange(n)
    in_band = explored = 0
    worst = dict(q=0.0, h=0.0, c=0.0, dq=0.0, dh=0.0, dc=0.0, mismatch_in_band=0)  # error / tolerance, max
    pv = orc.env_params_from_kwargs(**ENV_KW)
    P = orc.make_params(pv)
    names = ("x", "y", "vx", "vy", "spin", "top", "bot")
    finished = cut = long_traj = 0
    for k in range(nsteps):
        pre = _snap(L)
        L.step()
        post = _snap(L)
        aA = L.aA.cpu().numpy().astype(np.int64)
        aB = L.aB.cpu().numpy().astype(np.int64)
        # ---- acting vs the float64 oracle, from the device's carried (h, c), zeroed at episode start
        ctr, eps_k = pre["ctrl"]["step"], pre["ctrl"]["epsilon"]
        z = pre["reset"].astype(bool)
        hin = {s: pre[s].cpu().numpy().astype(np.float64) for s in ("hA", "cA", "hB", "cB")}
        for s in hin:
            hin[s][z] = 0.0
        # modelB: this step's fresh noise (reset_noise, :383-385) is the restated Philox draw, bit for
        # bit (the device's Box-Muller is a fixed sequence of correctly rounded operations)
        sdB = {kk: v.numpy() for kk, v in unpack_state_dict(L.learner.params).items()}
        for key, ref in orc.rnn_philox_noise(sp.seed_net, ctr).items():
            assert np.array_equal(sdB[key], ref), f"step {k}: {key}"
        qB_or, hB_or, cB_or = orc.rnn_forward(orc.rnn_effective(sdB, True), pre["obsB"][:, None, :], hin["hB"], hin["cB"])
        qA_or, hA_or, cA_or = np.empty_like(qB_or), np.empty_like(hB_or), np.empty_like(cB_or)
        for j, eff in enumerate(effA):
            sel = pre["opp"] == j
            if sel.any():
                qA_or[sel], hA_or[sel], cA_or[sel] = orc.rnn_forward(eff, pre["obsA"][sel][:, None, :], hin["hA"][sel],
                                                                     hin["cA"][sel])
        t = lambda x: x.cpu().numpy()  # noqa: E731
        ib, _, e1 = _check_rnn_act(f"step {k} A", aA, t(L.qA), t(post["hA"]), t(post["cA"]), qA_or, hA_or, cA_or,
                                   0.0, sp.seed_env, ctr, arenas, orc)
        in_band += ib
        ib, ex, e2 = _check_rnn_act(f"step {k} B", aB, t(L.qB), t(post["hB"]), t(post["cB"]), qB_or, hB_or, cB_or,
                                    eps_k, sp.seed_env, ctr, arenas, orc)
        in_band += ib
        explored += ex
        for kk in worst:
            worst[kk] = max(worst[kk], e1[kk], e2[kk]) if kk != "mismatch_in_band" else worst[kk] + e1[kk] + e2[kk]
        # ---- env tick on the oracle
        arr = np.zeros(n, orc.ARENA_DTYPE)
        for j, nm in enumerate(names):
            arr[nm] = pre["f64"][j]
        for j, nm in enumerate(("scoreA", "scoreB", "bounces")):
            arr[nm] = pre["i32"][j]
        oA, oB = orc.obs_of_arenas(arr)
        assert np.array_equal(oB, pre["obsB"]) and np.array_equal(oA, pre["obsA"])
        nA, nB, rew, done = orc.step_arenas(P, arr, aA.astype(np.int8), aB.astype(np.int8))
        d = done.astype(bool)
        e = d | (pre["es"] + 1 >= max_steps)  # episode end: done or the step cut
        rows = L.trans[k % L.depth].cpu().numpy()
        assert np.array_equal(rows[:, 0:7], oB) and np.array_equal(rows[:, 7], rew[:, 1])
        assert np.array_equal(rows[:, 8:15], nB)
        bits = rows[:, 15].view(np.int32)
        assert np.array_equal(bits & 0xFF, aB) and np.array_equal(bits >> 8, done.astype(np.int32))
        # ---- bookkeeping, next opponent, serve
        er = pre["er"] + rew[:, 1]
        ln = pre["el"] + 1
        ns = pre["i32"][3]
        q = orc.philox(np.arange(n), orc.TAG_OPP, ns, 0, sp.seed_env)
        use_pool = orc.u53(q[0], q[1]) < sp.pool_ratio
        newopp = np.where(use_pool, 1 + orc.below(q[2], L.n_pool), 0)
        vx, vy, spn = orc.philox_serve(pv, np.arange(n), ns, sp.seed_env)
        assert np.array_equal(post["opp"][e], newopp[e]) and np.array_equal(post["opp"][~e], pre["opp"][~e])
        assert np.all(post["er"][e] == 0) and np.array_equal(post["er"][~e], er[~e])
        assert np.all(post["el"][d] == 0) and np.array_equal(post["el"][~d], ln[~d])  # trajectory: done only
        assert np.all(post["es"][e] == 0) and np.array_equal(post["es"][~e], pre["es"][~e] + 1)
        assert np.array_equal(post["reset"].astype(bool), e)
        assert np.all(post["i32"][3][e] == ns[e] + 1) and np.array_equal(post["i32"][3][~e], ns[~e])
        assert np.array_equal(post["f64"][2][e], vx[e])
        assert np.array_equal(post["f64"][3][e], vy[e])
        assert np.array_equal(post["f64"][4][e], spn[e]) and np.all(post["f64"][0][e] == 0.5)
        for j, nm in enumerate(names):
            assert np.array_equal(post["f64"][j][~e], arr[nm][~e]), nm
        c0, c1 = pre["ctrl"], post["ctrl"]
        assert c1["step"] == c0["step"] + 1 and c1["episodes"] == c0["episodes"] + e.sum()
        assert c1["ep_A"] - c0["ep_A"] == (e & (pre["opp"] == 0)).sum()
        assert c1["win_A"] - c0["win_A"] == (e & (pre["opp"] == 0) & (er > 0)).sum()
        assert c1["ep_P"] - c0["ep_P"] == (e & (pre["opp"] != 0)).sum()
        assert c1["seq_count"] - c0["seq_count"] == (d & (ln >= L.T)).sum()
        finished += int(d.sum())
        cut += int((e & ~d).sum())
        long_traj = max(long_traj, int(ln[d].max()) if d.any() else 0)
    print(f"\nrnn act vs oracle, n={n} eps={eps}: {2 * n * nsteps} decisions, {in_band} greedy ones in the "
          f"tie band (either near-max accepted; {worst['mismatch_in_band']} of them differ from the oracle's argmax), "
          f"{explored} epsilon-branch ones exact; max error / tolerance q {worst['q']:.3f} h {worst['h']:.3f} "
          f"c {worst['c']:.3f}; max abs error q {worst['dq']:.2e} h {worst['dh']:.2e} c {worst['dc']:.2e}")
    assert in_band <= 2 * n * nsteps // 100  # the band is rare (< 1 % of decisions)
    if eps > 0:
        assert explored > 0.2 * eps * n * nsteps
    assert finished > (50 if max_steps == 1000 else 10)  # episodes did end and restart during the run
    if max_steps < 1000:
        assert cut > 100 and long_traj > max_steps  # cuts happened; a stored trajectory spanned a cut
    else:
        assert cut == 0
    assert L.counters()["train_steps"] == 0


def test_rnn_sequence_buffer_and_training(golden):
    T, B, cap = 8, 64, 3000
    L = _learner(golden, n=2048, n_pool=2, epsilon=1.0, min_epsilon=0.05, epsilon_decay=0.999, memory_size=cap,
                 min_episodes_for_training_start=1, seed=11)
    trained = 0
    for k in range(140):
        L.step()
        c = L.counters()
        trained += c["train"]
        assert c["train"] == int(c["seq_size"] > B), f"step {k}"
        assert c["train_steps"] == trained
    c = L.counters()
    assert c["status"] == 0 and c["seq_count"] > cap and c["seq_size"] == cap  # wrapped around
    assert c["episodes"] == c["ep_A"] + c["ep_P"] and c["seq_count"] <= c["episodes"]
    eps = 1.0
    for _ in range(c["episodes"]):
        eps = max(0.05, eps * 0.999)
    assert c["epsilon"] == eps
    st = L.learner.stats()
    assert trained > 50 and st["steps"] == trained and np.isfinite(st["loss"]) and st["norm"] > 0
    # every stored episode: one contiguous trajectory in its arena's ring, done only on its last step
    ring = L.trans.cpu().numpy()
    eps_tab = L.episodes().numpy()
    assert len(eps_tab) == cap
    now = c["step"]
    for arena, start, length in eps_tab[::7]:
        assert length >= T and start + length - 1 <= now - 1 and now - 1 - start < L.depth
        rec = ring[(start + np.arange(length)) % L.depth, arena]
        bits = rec[:, 15].view(np.int32)
        assert np.all(bits[:-1] >> 8 == 0) and bits[-1] >> 8 == 1
        assert np.array_equal(rec[1:, 0:7], rec[:-1, 8:15])  # next_obs[t] == obs[t+1]
    # the sampled batch: windows of stored episodes
    obs, nxt = L.learner.obs.cpu().numpy(), L.learner.next.cpu().numpy()
    done = L.learner.done.cpu().numpy()
    assert np.array_equal(obs[:, 1:], nxt[:, :-1]) and np.all(done[:, :-1] == 0)


def test_rnn_selfplay_deterministic(golden):
    runs = []
    for _ in range(2):
        L = _learner(golden, n=1024, n_pool=1, epsilon=0.5, memory_size=2000, min_episodes_for_training_start=1,
                     seed=4)
        for _ in range(60):
            L.step()
        runs.append((L.learner.params.clone(), L.trans.clone(), L.counters()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1]) and runs[0][2] == runs[1][2]


def test_two_ranks_stay_identical(golden):
    """world = 2 on one device: each rank its own arenas / buffer (rank-specific env seed), the
    gradients (+ rank count) summed as the all-reduce would, the same Adam step on both."""
    from pongmi.rnn_selfplay import RNNSelfPlayLearner
    g = golden("rnn")
    Ls = [RNNSelfPlayLearner(ENV_KW, 1024, _golden_sd(g), _rnn_sd(7), [], epsilon=0.5, memory_size=2000,
                             min_episodes_for_training_start=1, seed=9, rank=r, world=2, allreduce=lambda t: None)
          for r in range(2)]
    both = 0
    for _ in range(70):
        for L in Ls:
            L.rollout()
            L.learner.grads()
        s = Ls[0].learner.grad + Ls[1].learner.grad
        ranks = s[-4].item()
        for L in Ls:
            L.learner.grad.copy_(s)
            L.learner.apply()
        both += ranks == 2
        assert torch.equal(Ls[0].learner.params, Ls[1].learner.params)
    assert both > 10
    assert not torch.equal(Ls[0].trans, Ls[1].trans)  # different arenas per rank
    assert Ls[0].learner.stats()["steps"] == Ls[1].learner.stats()["steps"] > 0


def test_rnn_ring_safety(golden):
    """A ring too shallow for the episodes (depth 64: trajectories up to 32 steps, episodes leave
    the buffer 32 steps after they finish): nothing a sample reads was overwritten (status bit 0
    never set), every held episode is intact in its ring, long trajectories are dropped (bit 2) and
    age eviction is reported (bit 1); check_status raises only on bit 0."""
    from pongmi import _lib
    L = _learner(golden, n=512, n_pool=1, epsilon=0.3, memory_size=100_000, min_episodes_for_training_start=1,
                 seed=6, depth=64)
    for _ in range(150):
        L.step()
    c = L.counters()
    assert c["status"] & 1 == 0 and c["status"] & 2 and c["seq_size"] < c["seq_count"] < 100_000
    now = c["step"]
    ring = L.trans.cpu().numpy()
    for arena, start, length in L.episodes().numpy():
        assert _storable(length, L) and now - 1 - start < L.depth
        rec = ring[(start + np.arange(length)) % L.depth, arena]
        bits = rec[:, 15].view(np.int32)
        assert np.all(bits[:-1] >> 8 == 0) and bits[-1] >> 8 == 1
    msgs = []
    L.check_status(log=msgs.append)
    assert any("evicted" in m for m in msgs)
    L.set_counters(status=1)
    with pytest.raises(_lib.PongmiError):
        L.check_status(log=msgs.append)


def _storable(length, L):
    return L.T <= length <= L.depth // 2


def test_rnn_updates_per_step(golden):
    """U = 3 DRQN updates per vector step, each on its own batch (Philox counter (step, u)): the fused
    pm_rnn_selfplay_step_multi equals rollout + update + (sample(u) + update) x 2 bit for bit, and
    train steps advance by U per enabled step."""
    U = 3
    A = _learner(golden, n=1024, n_pool=1, epsilon=0.5, memory_size=2000, min_episodes_for_training_start=1, seed=4,
                 updates_per_step=U)
    B = _learner(golden, n=1024, n_pool=1, epsilon=0.5, memory_size=2000, min_episodes_for_training_start=1, seed=4)
    enabled = 0
    for _ in range(50):
        A.step()
        B.rollout()
        B.learner.update()
        obs0 = B.learner.obs.clone()
        for u in range(1, U):
            B.sample(u)
            if B.counters()["train"]:
                assert not torch.equal(B.learner.obs, obs0)  # a fresh batch per update
            B.learner.update()
        enabled += B.counters()["train"]
    torch.cuda.synchronize()
    assert torch.equal(A.learner.params, B.learner.params) and torch.equal(A.trans, B.trans)
    assert A.counters() == B.counters()
    assert enabled > 10 and A.learner.stats()["steps"] == U * enabled


@pytest.mark.parametrize("U", [1, 2])
def test_rnn_overlapped_step_is_bitwise_identical(golden, U):
    """pm_rnn_selfplay_step_overlap (the next step's opponent act on a side stream beside the DRQN
    update, modelB's act only in the step) against the plain step: every state, action, ring record,
    parameter and counter equal, also across a pool model added and a modelA swap mid-run."""
    from pongmi import _lib
    kw = dict(n=1024, n_pool=2, epsilon=0.3, memory_size=2000, min_episodes_for_training_start=1, seed=6,
              updates_per_step=U)
    A = _learner(golden, overlap=False, **kw)
    B = _learner(golden, overlap=True, **kw)
    for k in range(60):
        if k == 25:
            for L in (A, B):
                L.add_pool_model(_rnn_sd(300))
        if k == 40:
            for L in (A, B):
                L.set_modelA(_rnn_sd(301))
        A.step()
        B.step()
        if k % 10 == 9:
            sa, sb = _snap(A), _snap(B)
            for key in sa:
                if key in ("hA", "cA"):  # B's opponent side is already one act ahead (the next step's)
                    continue
                if key == "ctrl":
                    assert sa[key] == sb[key], k
                elif isinstance(sa[key], torch.Tensor):
                    assert torch.equal(sa[key], sb[key]), (k, key)
                else:
                    assert np.array_equal(sa[key], sb[key]), (k, key)
    A.act_part(_lib.PM_ACT_A)  # A's opponents act for the current observations, as B's already did
    torch.cuda.synchronize()
    assert torch.equal(A.learner.params, B.learner.params)
    assert torch.equal(A.trans, B.trans) and torch.equal(A.aA, B.aA) and torch.equal(A.aB, B.aB)
    assert torch.equal(A.hA, B.hA) and torch.equal(A.cA, B.cA)
    assert A.learner.stats()["steps"] == B.learner.stats()["steps"] > 0


@pytest.mark.parametrize("split_r", ["0", "3"])
def test_rnn_split_tiles_are_bitwise_identical(golden, monkeypatch, split_r):
    """The overlapped step's side-A act with its groups from `split_r` on run as split tiles
    (rnn_tile_split: one 32-arena tile per block, the ring's four pieces on the four waves; forced
    with PONGMI_RNN_SPLIT_R, "0" = every group) equals the same step with splitting off
    (PONGMI_RNN_SPLIT=0): opponents' actions, q-driven decisions, (h, c), ring records, modelB."""
    kw = dict(n=1024, n_pool=3, epsilon=0.3, memory_size=2000, min_episodes_for_training_start=1, seed=8)
    A = _learner(golden, overlap=True, **kw)
    B = _learner(golden, overlap=True, **kw)
    for k in range(30):
        if k == 20:
            for L in (A, B):
                L.set_modelA(_rnn_sd(302))
        monkeypatch.setenv("PONGMI_RNN_SPLIT", "0")
        A.step()
        monkeypatch.delenv("PONGMI_RNN_SPLIT")
        monkeypatch.setenv("PONGMI_RNN_SPLIT_R", split_r)
        B.step()
        monkeypatch.delenv("PONGMI_RNN_SPLIT_R")
    torch.cuda.synchronize()
    assert torch.equal(A.hA, B.hA) and torch.equal(A.cA, B.cA) and torch.equal(A.aA, B.aA)
    assert torch.equal(A.learner.params, B.learner.params) and torch.equal(A.trans, B.trans)
    assert A.counters() == B.counters() and A.learner.stats()["steps"] > 0


@pytest.mark.parametrize("change", [None, "modelA"])
def test_rnn_split_step_after_overlapped_steps(golden, change):
    """The generation controller's save-boundary step (rollout + updates, pongmi.generations
    RNNGenerations._step) between overlapped steps, optionally after a modelA swap: the opponents'
    (h, c) and actions, modelB's state and every counter equal an uninterrupted plain run (the
    opponents' LSTM must advance exactly once per observation: ADVICE r2)."""
    kw = dict(n=1024, n_pool=2, epsilon=0.3, memory_size=2000, min_episodes_for_training_start=1, seed=9)
    A = _learner(golden, overlap=True, **kw)
    B = _learner(golden, overlap=False, **kw)
    for k in range(30):
        if change and k == 17:
            for L in (A, B):
                L.set_modelA(_rnn_sd(305))
        B.step()
        if k in (12, 17, 18):  # the controller's split step (save boundary)
            A.rollout()
            A.learner.update()
        else:
            A.step()
    sa, sb = _snap(A), _snap(B)
    for key in sa:
        if key in ("hA", "cA"):
            continue  # A's opponents are one (speculative) act ahead after an overlapped step
        if key == "ctrl":
            assert sa[key] == sb[key]
        elif isinstance(sa[key], torch.Tensor):
            assert torch.equal(sa[key], sb[key]), key
        else:
            assert np.array_equal(sa[key], sb[key]), key
    from pongmi import _lib
    B.act_part(_lib.PM_ACT_A)  # B's opponents act for the current observations, as A's speculative act did
    torch.cuda.synchronize()
    assert torch.equal(A.hA, B.hA) and torch.equal(A.cA, B.cA) and torch.equal(A.aA, B.aA)
    assert torch.equal(A.learner.params, B.learner.params) and torch.equal(A.trans, B.trans)
    assert A.learner.stats()["steps"] == B.learner.stats()["steps"] > 0


def test_rnn_production_step_equals_plain_at_full_size(golden):
    """configs[4] at its full size (the bench's workload: 32 768 arenas, pool 4, sequence buffer
    200 000, DRQN 64 x 8 every step once the buffer holds enough episodes): the overlapped production
    step equals the plain step bit for bit through the start of training."""
    from pongmi import _lib
    kw = dict(n=32768, n_pool=4, epsilon=0.05, seed=7)
    A = _learner(golden, overlap=False, **kw)
    B = _learner(golden, overlap=True, **kw)
    for _ in range(40):
        A.step()
        B.step()
    A.act_part(_lib.PM_ACT_A)  # A's opponents act for the current observations, as B's already did
    torch.cuda.synchronize()
    assert torch.equal(A.learner.params, B.learner.params)
    assert torch.equal(A.trans, B.trans) and torch.equal(A.aA, B.aA) and torch.equal(A.aB, B.aB)
    assert torch.equal(A.hA, B.hA) and torch.equal(A.cA, B.cA) and torch.equal(A.hB, B.hB)
    assert A.counters() == B.counters()
    assert A.learner.stats()["steps"] == B.learner.stats()["steps"] > 0
