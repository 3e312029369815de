"""K5 — QNetRNN on the matrix cores (pm_rnn_fold / pm_rnn_q / pm_rnn_act) against the reference's
own outputs (tests/golden/rnn.npz, produced by models/qnet_rnn.py on checkpoints_rnn/rnn_pong_soul_3.pth)
and the float64 oracle (oracle.rnn_forward).

Tolerance: the kernel computes in fp32 (exact-f32 MFMA, a different summation order than torch's
CPU GEMMs); Q / h / c agree with the reference to rtol 1e-4, atol 1e-5 (|values| <= ~5) over one
step, the 8-step sequence and the 12-step carried roll-out. Integer actions: identical to the
argmax (first max) of the same kernel's Q values; the two entry points (pm_rnn_q, pm_rnn_act)
are bit-identical on the same rows.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-4, 1e-5


def _sd(g):
    return {k[7:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("params.")}


def _w(g, mode):
    from pongmi import _lib, rnn
    m = _lib.PM_FOLD_TRAIN if mode == "train" else _lib.PM_FOLD_EVAL
    return rnn.fold(rnn.pack_state_dict(_sd(g)), m)[0]


def _close(a, b, what):
    np.testing.assert_allclose(a.detach().cpu().numpy() if torch.is_tensor(a) else a, b, rtol=RTOL, atol=ATOL,
                               err_msg=what)


@pytest.mark.parametrize("mode", ["train", "eval"])
def test_rnn_step_matches_reference(golden, mode):
    from pongmi import rnn
    g = golden("rnn")
    w = _w(g, mode)
    h = torch.from_numpy(g["act_h0"][0]).cuda().contiguous()
    c = torch.from_numpy(g["act_c0"][0]).cuda().contiguous()
    q = rnn.q_step(w, torch.from_numpy(g["act_x"][:, 0]).cuda(), h, c)
    _close(q, g[f"act_q_{mode}"], "q")
    _close(h, g[f"act_h1_{mode}"][0], "h")
    _close(c, g[f"act_c1_{mode}"][0], "c")


@pytest.mark.parametrize("mode", ["train", "eval"])
def test_rnn_sequence_matches_reference(golden, mode):
    from pongmi import rnn
    g = golden("rnn")
    q, h, c = rnn.forward(_w(g, mode), torch.from_numpy(g["seq_x"]).cuda())
    _close(q, g[f"seq_q_{mode}"], "q")
    _close(h, g[f"seq_h_{mode}"][0], "h")
    _close(c, g[f"seq_c_{mode}"][0], "c")


def test_rnn_rollout_matches_reference(golden):
    """12 acting steps with the state carried (select_action_for_model, train_rnn_iterative.py:371-389)."""
    from pongmi import rnn
    g = golden("rnn")
    w = _w(g, "train")
    h, c = rnn.init_state(16)
    for t in range(12):
        q = rnn.q_step(w, torch.from_numpy(g["roll_x"][t]).cuda(), h, c)
        _close(q, g["roll_q"][t], f"q at step {t}")
    _close(h, g["roll_h"][0], "h")
    _close(c, g["roll_c"][0], "c")


def test_dropin_module_matches_reference(golden):
    """models.qnet_rnn.QNetRNN on the device (HIP path) and with autograd (torch path)."""
    from models.qnet_rnn import QNetRNN
    g = golden("rnn")
    net = QNetRNN(7, 3).cuda()
    net.load_state_dict(_sd(g))
    x = torch.from_numpy(g["seq_x"]).cuda()
    for mode in ("train", "eval"):
        net.train(mode == "train")
        with torch.no_grad():
            q, (h, c) = net(x, net.init_hidden(16, "cuda"))
        assert h.shape == (1, 16, 128) and c.shape == (1, 16, 128)
        _close(q, g[f"seq_q_{mode}"], "q (HIP path)")
        _close(h[0], g[f"seq_h_{mode}"][0], "h (HIP path)")
    net.train(True)
    q, _ = net(x, net.init_hidden(16, "cuda"))  # autograd: the torch path
    assert q.requires_grad
    _close(q, g["seq_q_train"], "q (torch path)")


def test_rnn_against_oracle_random_states(golden, orc):
    """4096 rows of random observations and warm states against the float64 oracle."""
    from pongmi import rnn
    g = golden("rnn")
    sd = {k[7:]: v for k, v in g.items() if k.startswith("params.")}
    rng = np.random.default_rng(11)
    n = 4096
    x = rng.uniform(-1, 1, (n, 7)).astype(np.float32)
    x[:, 6] *= 5
    h0 = rng.normal(0, 0.4, (n, 128)).astype(np.float32)
    c0 = rng.normal(0, 0.8, (n, 128)).astype(np.float32)
    for mode in ("train", "eval"):
        h, c = torch.from_numpy(h0).cuda(), torch.from_numpy(c0).cuda()
        q = rnn.q_step(_w(g, mode), torch.from_numpy(x).cuda(), h, c)
        eff = orc.rnn_effective(sd, mode == "train")
        qo, ho, co = orc.rnn_forward(eff, x[:, None, :], h0, c0)
        # fp32 vs float64 on warm random states (pre-activations up to ~20): one fp32 K = 256 gate
        # dot product carries ~256 * 2^-24 * sum|w x| of rounding, up to ~2e-5 on c
        for a, b, what in ((q, qo, "q"), (h, ho, "h"), (c, co, "c")):
            np.testing.assert_allclose(a.cpu().numpy(), b, rtol=RTOL, atol=5e-5, err_msg=what)


def test_rnn_reset_rows_start_from_zero(golden):
    from pongmi import rnn
    g = golden("rnn")
    w = _w(g, "train")
    n = 300  # ragged: not a multiple of the 32-arena tile or the 128-row block
    rng = np.random.default_rng(3)
    x = torch.from_numpy(rng.uniform(0, 1, (n, 7)).astype(np.float32)).cuda()
    h0 = torch.from_numpy(rng.normal(0, 0.4, (n, 128)).astype(np.float32)).cuda()
    c0 = torch.from_numpy(rng.normal(0, 0.8, (n, 128)).astype(np.float32)).cuda()
    reset = torch.from_numpy(rng.random(n) < 0.3).cuda()
    h, c = h0.clone(), c0.clone()
    q = rnn.q_step(w, x, h, c, reset=reset)
    hz, cz = h0.clone(), c0.clone()
    hz[reset] = 0
    cz[reset] = 0
    q2 = rnn.q_step(w, x, hz, cz)
    assert torch.equal(q, q2) and torch.equal(h, hz) and torch.equal(c, cz)


def _host_lists(opp, nn):
    """Per-256-arena-block opponent lists as the env kernels write them (write_opp_lists)."""
    n = len(opp)
    neb = (n + 255) // 256
    lst = np.zeros(n, np.int32)
    cnt = np.zeros(neb * nn, np.int32)
    for e in range(neb):
        ids = opp[e * 256:(e + 1) * 256]
        off = 0
        for k in range(nn):
            sel = np.nonzero(ids == k)[0] + e * 256
            lst[e * 256 + off:e * 256 + off + len(sel)] = sel
            cnt[e * nn + k] = (off << 16) | len(sel)
            off += len(sel)
    return lst, cnt


@pytest.mark.parametrize("n,n_opp,lists", [(1000, 1, False), (5000, 3, False), (257, 9, False), (5000, 3, True),
                                           (33000, 5, True), (300, 9, True)])
def test_rnn_act_matches_q_step(golden, n, n_opp, lists):
    """The fused two-player act: A greedy with its opponent's net, B greedy (eps = 0) — actions are
    the first-max argmax of the same Q values pm_rnn_q returns, states advance identically."""
    from pongmi import _lib, rnn
    from models.qnet_rnn import QNetRNN
    g = golden("rnn")
    wB = _w(g, "train")
    torch.manual_seed(7)
    nets = [QNetRNN(7, 3) for _ in range(n_opp)]
    w_opp = rnn.fold(torch.stack([rnn.pack_state_dict(m.state_dict()) for m in nets]), _lib.PM_FOLD_EVAL)
    rng = np.random.default_rng(n)
    obsA = torch.from_numpy(rng.uniform(0, 1, (n, 7)).astype(np.float32)).cuda()
    obsB = torch.from_numpy(rng.uniform(0, 1, (n, 7)).astype(np.float32)).cuda()
    opp = torch.from_numpy(rng.integers(0, n_opp, n).astype(np.int32)).cuda() if n_opp > 1 else None
    stA = [torch.from_numpy(rng.normal(0, 0.4, (n, 128)).astype(np.float32)).cuda() for _ in range(2)]
    stB = [torch.from_numpy(rng.normal(0, 0.4, (n, 128)).astype(np.float32)).cuda() for _ in range(2)]
    refA = [t.clone() for t in stA]
    refB = [t.clone() for t in stB]
    kw = {}
    if lists:  # side A packed over per-block lists (the self-play loop's path)
        oid_h = opp.cpu().numpy() if opp is not None else np.zeros(n, np.int32)
        if opp is None:
            opp = torch.zeros(n, dtype=torch.int32, device="cuda")
        lst, cnt = _host_lists(oid_h, n_opp)
        kw = dict(opp_list=torch.from_numpy(lst).cuda(), opp_cnt=torch.from_numpy(cnt).cuda())
    aA, aB, qA, qB = rnn.act(w_opp, opp, wB, obsA, obsB, stA, stB, epsilon=0.0, want_q=True, chunk1=1024, **kw)
    qB_ref = rnn.q_step(wB, obsB, *refB)
    qA_ref = torch.empty_like(qA)
    hA, cA = torch.empty_like(refA[0]), torch.empty_like(refA[1])
    oid = opp.long() if opp is not None else torch.zeros(n, dtype=torch.long, device="cuda")
    for k in range(n_opp):
        sel = (oid == k).nonzero().flatten()
        if sel.numel() == 0:
            continue
        hk, ck = refA[0][sel].contiguous(), refA[1][sel].contiguous()
        qA_ref[sel] = rnn.q_step(w_opp[k], obsA[sel], hk, ck)
        hA[sel], cA[sel] = hk, ck
    assert torch.equal(qB, qB_ref) and torch.equal(qA, qA_ref)
    assert torch.equal(stB[0], refB[0]) and torch.equal(stB[1], refB[1])
    assert torch.equal(stA[0], hA) and torch.equal(stA[1], cA)
    assert torch.equal(aB.long(), qB.argmax(1)) and torch.equal(aA.long(), qA.argmax(1))


def test_rnn_act_epsilon_and_reset(golden):
    """eps = 1: B acts uniformly at random in {0, 1, 2} but its forward still advances (h, c)
    (train_rnn_iterative.py:379-383); reset zeroes both players' state first."""
    from pongmi import rnn
    g = golden("rnn")
    w = _w(g, "train")
    n = 4096
    rng = np.random.default_rng(1)
    obs = torch.from_numpy(rng.uniform(0, 1, (n, 7)).astype(np.float32)).cuda()
    st = [torch.from_numpy(rng.normal(0, 0.4, (n, 128)).astype(np.float32)).cuda() for _ in range(4)]
    reset = torch.zeros(n, dtype=torch.bool, device="cuda")
    reset[::5] = True
    ref = [t.clone() for t in st]
    for t in ref:
        t[reset] = 0
    pre = [t.clone() for t in ref]
    aA, aB = rnn.act(w.reshape(1, -1), None, w, obs, obs, st[:2], st[2:], reset=reset, epsilon=1.0, seed=5, counter=9)
    qA = rnn.q_step(w, obs, ref[0], ref[1])
    qB = rnn.q_step(w, obs, ref[2], ref[3])
    for a, b in zip(st, ref):
        assert torch.equal(a, b)
    assert torch.equal(aA.long(), qA.argmax(1))
    counts = torch.bincount(aB.long(), minlength=3).cpu().numpy()
    assert counts.min() > n / 3 - 5 * np.sqrt(n * 2 / 9), counts
    assert (aB.long() != qB.argmax(1)).any()
    aA2, aB2 = rnn.act(w.reshape(1, -1), None, w, obs, obs, pre[:2], pre[2:], epsilon=1.0, seed=5, counter=9)
    assert torch.equal(aB, aB2)  # Philox(seed, counter): reproducible


def test_rnn_fold_fresh_noise_writes_buffers(golden):
    """train_fresh: reset_noise() on the device (factorised Gaussian, models/qnet_rnn.py:33-41) —
    weight_epsilon = outer(f(e_out), f(e_in)), bias_epsilon = f(e_out), written back, and the
    folded weights equal a train-mode fold of the written-back block."""
    from pongmi import _lib, rnn
    g = golden("rnn")
    p = rnn.pack_state_dict(_sd(g))
    out = p.clone()
    w = rnn.fold(p, _lib.PM_FOLD_TRAIN_FRESH, seed=3, counter=4, params_out=out)[0]
    sd = rnn.unpack_state_dict(out)
    for m in ("fc_shared_head.0", "fc_V", "fc_A"):
        we, be = sd[f"{m}.weight_epsilon"], sd[f"{m}.bias_epsilon"]
        assert not torch.equal(be, torch.from_numpy(g[f"params.{m}.bias_epsilon"]))
        r = int(be.abs().argmax())
        e_in = we[r] / be[r]
        torch.testing.assert_close(we, torch.outer(be, e_in), rtol=1e-5, atol=1e-6)
    assert torch.equal(rnn.fold(out, _lib.PM_FOLD_TRAIN)[0], w)
    w2 = rnn.fold(p, _lib.PM_FOLD_TRAIN_FRESH, seed=3, counter=5)[0]
    assert not torch.equal(w, w2)
